set -e
for d in 0 1; do for pf in "" "--no-prefetch"; do echo "describe2=$d $pf"; timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --opt describe2=$d $pf 2>&1 | grep -o '"value": [0-9.]*\|host_ms.*' | tr '\n' ' '; echo; done; done
