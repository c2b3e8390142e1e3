set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_round.sh ${TAG:-r02g} tests bench fif1 c2c5 prof || exit $?
for cfg in bunny:full bunny:primary; do
  IFS=: read sc mode <<< "$cfg"
  timeout -k 10 200 python bench.py --scene $sc --mode $mode --frames-in-flight 1 --no-cpu --steps 100 --warmup 5 \
      > gpurun_out/${TAG:-r02g}/bench_${sc}_${mode}_fif1.json 2> gpurun_out/${TAG:-r02g}/bench_${sc}_${mode}_fif1.err
  rc=$?; echo "$sc $mode fif1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
