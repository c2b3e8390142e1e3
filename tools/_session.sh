SWEEP="0:4 1:4" RUN_TESTS=1 bash tools/sweep.sh
