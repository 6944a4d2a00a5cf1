set -e
for e in 0 1; do for r in 0 32; do echo "early=$e reserve=$r"; timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --side-cu-reserve $r --prefetch-early $e 2>&1 | grep -o '"value": [0-9.]*\|host_ms.*' | tr '\n' ' '; echo; done; done
