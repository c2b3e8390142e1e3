set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ep
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ep/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ep/pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=ep LIBS="default ep0" CFGS="soup:primary:1 soup:primary:4 bunny:primary:4 bunny:full:4 soup:full:4" REPS=2 bash tools/ablibs.sh
