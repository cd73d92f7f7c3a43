set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r1final SKIP_TESTS=0 bash tools/gpu_check.sh || exit $?
TAG=r1final_pmc PMC_GROUPS="FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES__GRBM_GUI_ACTIVE__SQ_WAVE_CYCLES__SQ_WAIT_ANY__SQ_BUSY_CYCLES" bash tools/pmc.sh || exit $?
mkdir -p gpurun_out/r1final_c3 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1final_c3/prof -o c3 -- python bench.py --config c3 --steps 10 --warmup 3 > gpurun_out/r1final_c3/c3prof.log 2>&1 && timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 > gpurun_out/r1final_c3/c3.log 2>&1 && timeout -k 10 300 python bench.py --config c4 --no-fp32-run > gpurun_out/r1final_c3/c4.log 2>&1
echo "all rc=$?"
