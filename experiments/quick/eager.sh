# which side faults when HIP loads every code object at start-up
# (HIP_ENABLE_DEFERRED_LOADING=0)? Steps from the smallest process up; the first failing step ends
# the call (no GPU work after a fault). faulthandler prints the Python stack of a segfault.
export HIP_ENABLE_DEFERRED_LOADING=0
mkdir -p gpurun_out
step() {
  name=$1; shift
  echo "== $name: $*"
  timeout -k 10 180 "$@" > gpurun_out/eager_$name.log 2>&1
  rc=$?
  echo "rc=$rc"
  tail -25 gpurun_out/eager_$name.log
  [ $rc -eq 0 ] || exit 0
}
step hipinfo python3 -c "import ctypes; h=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so'); n=ctypes.c_int(); print('system HIP devices', h.hipGetDeviceCount(ctypes.byref(n)), n.value)"
step headless ./b-shot-slam_amd/bin/odometry_headless 3 600 0
step torch python3 -X faulthandler -c "import torch; x=torch.zeros(4, device='cuda'); print('torch ok', float(x.sum()))"
step lib python3 -X faulthandler -c "import sys; sys.path.insert(0, 'b-shot-slam_amd'); import bshot_py; c = bshot_py.Context(0); pc, _ = bshot_py.synth_sweep(0); c.set_cloud(pc); print('lib ok', c.seg_ratio()[:3])"
step bench python3 -X faulthandler bench.py --no-cpu-baseline --no-upload-leg --steps 20 --warmup 5
echo "every step ran"
