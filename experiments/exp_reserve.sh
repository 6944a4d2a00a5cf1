set -e
HT_TIMEOUT=30 timeout -k 5 40 python -u b-shot-slam_amd/tools/sr_variants.py 4,0 4,0 | cut -c1-60
for r in 0 16 32 64; do echo "reserve=$r"; timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --side-cu-reserve $r 2>&1 | grep -o '"value": [0-9.]*\|host_ms.*' | tr '\n' ' '; echo; done
