set -e
for cfg in "2 0" "4 0" "2 1" "4 1"; do set -- $cfg; echo "ladder=$1 hint=$2"; timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --ladder-grids $1 --sr-hint $2 2>&1 | grep -o '"value": [0-9.]*\|"grid": [0-9.]*\|"seg_ratio": [0-9.]*' | tr '\n' ' '; echo; done
