set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kn
timeout -k 10 300 python -u -m pytest tests/test_gpu_kilonerf.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/kn/tests.log 2>&1; rc=$?; tail -3 gpurun_out/kn/tests.log; [ $rc -eq 0 ] || exit $rc
if [ -e nerf-rep_for_test_amd/lib/libnerfhip_old.so ]; then
  NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_old.so timeout -k 10 300 python tools/hbm_bench.py gpurun_out/kn/hbm_old.json > gpurun_out/kn/hbm_old.log 2>&1 || exit $?
fi
timeout -k 10 300 python tools/hbm_bench.py gpurun_out/kn/hbm_new.json > gpurun_out/kn/hbm_new.log 2>&1 || exit $?
grep -h "kn_" gpurun_out/kn/hbm_*.log | cut -c1-170
