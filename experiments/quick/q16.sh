set -u
O=gpurun_out; mkdir -p $O
echo "[q16] $(date +%T) pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu_r02i.log 2>&1; rc=$?
tail -2 $O/pytest_gpu_r02i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r02i.log 2>&1 && tail -1 $O/smoke_r02i.log || exit 1
bash scripts/q15.sh
