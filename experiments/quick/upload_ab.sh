# upload leg run after the main leg's odometry is closed
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/up_$r.json 2>gpurun_out/up_$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/up_$r.json')); print('run $r', 'value', d['value'], 'upload leg', d['upload_inclusive']['value'])"
done
