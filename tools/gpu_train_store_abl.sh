set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl2
for v in base nostore zerorec base nostore zerorec; do
  if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/time_train_fwd.py 196608 20 2>&1 | tail -3 || exit $?
done
