set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for tag in default pk; do
  if [ $tag = default ]; then lib=""; else lib=$PWD/ray-tracing-project_amd/lib/librtamd_pk.so; fi
  RTAMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS} -d gpurun_out/pkprof${PASS:-}/$tag -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu --no-side --no-extra --no-e2e > gpurun_out/pkprof${PASS:-}/$tag.log 2>&1 || exit 1
done
