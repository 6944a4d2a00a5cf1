# A/B of the tree's library against a `make variant` build, alternating on one box.
# usage: bash experiments/quick/ab_variant.sh <variant .so> <rounds>
V=$1; N=${2:-3}
O=gpurun_out; mkdir -p $O
for L in b-shot-slam_amd/lib/libbshot_amd.so $V; do BSHOT_LIB=$(pwd)/$L timeout -k 10 100 python b-shot-slam_amd/tools/sr_bench.py 2>/dev/null | grep lib; done
for i in $(seq 1 $N); do for L in b-shot-slam_amd/lib/libbshot_amd.so $V; do
  BSHOT_LIB=$(pwd)/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg > $O/abv_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/abv_$i.json')); print('$L', $i, d['value'], d['ms_per_step_median'], d['stage_ms_per_sweep'].get('seg_ratio'))"
done; done
