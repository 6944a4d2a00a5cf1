set -e
for r in 0 16 32 64; do echo "reserve=$r"; timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --side-cu-reserve $r 2>&1 | grep -o '"value": [0-9.]*\|"match": [0-9.]*\|"seg_ratio": [0-9.]*\|host_ms.*' | tr '\n' ' '; echo; done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-prefetch | grep -o '"value": [0-9.]*'
