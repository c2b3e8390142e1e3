#!/bin/bash
# Round-6 GPU pass: GPU tests (product library, and the RT_CHECK_PREFETCH debug build), the default bench
# line, the in-process multi-device line rehearsed on one GPU, rocprofv3 profiles of the headline kernel (C3)
# and of the C5 / C2 kernels, and the round's A/B measurements. Every GPU step has its own time limit; stop at
# the first hard failure.
# Usage: bash tools/gpu_round6.sh <tag> [tests pftests bench multi prof profc5 profc2 moving ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift || true
STEPS=${*:-tests bench prof profc5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
hard() { case $1 in 124|134|137|139) echo "hard failure ($1): stopping"; exit $1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
          --durations=15 > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log; hard $rc ;;
    pftests)
      # the whole GPU suite against the debug build whose kernels check every scalar prefetch offset
      RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_pfcheck.so timeout -k 10 600 python -u -m pytest tests -m gpu -q \
          -p no:cacheprovider --timeout 300 --timeout-method thread \
          --deselect tests/test_gpu_parity.py::test_product_library_refuses_variant_only_kernels > $OUT/pytest_gpu_pfcheck.log 2>&1
      rc=$?; echo "pfcheck pytest rc=$rc"; tail -8 $OUT/pytest_gpu_pfcheck.log; hard $rc ;;
    mdtests)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_multidevice.py -q -p no:cacheprovider --timeout 200 \
          --timeout-method thread > $OUT/pytest_md.log 2>&1
      rc=$?; echo "multidevice pytest rc=$rc"; tail -5 $OUT/pytest_md.log; hard $rc ;;
    moving)
      # lone frames under the moving camera: this library's longest-first policies, and the round-5 library
      # (per-slot cost maps) when lib/librtamd_r05.so was built beside it (tools/moving_ab.py)
      export RTAMD_DEBUG_KNOBS=1
      for sc in ${MSCENES:-soup:primary bunny:full}; do
        IFS=: read scn md <<< "$sc"
        for pol in ${MPOLICIES:-lib moved0 r1 nolpt}; do
          timeout -k 10 180 python tools/moving_ab.py $scn $md $pol 60 2 >> $OUT/moving.jsonl 2>> $OUT/moving.err
          rc=$?; [ $rc -ne 0 ] && { echo "moving $scn $pol rc=$rc"; hard $rc; exit $rc; }
        done
        if [ -f ray-tracing-project_amd/lib/librtamd_r05.so ] && [ -z "${MNOR05:-}" ]; then
          RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_r05.so timeout -k 10 180 python tools/moving_ab.py $scn $md lib 60 2 \
              >> $OUT/moving.jsonl 2>> $OUT/moving.err
          rc=$?; [ $rc -ne 0 ] && { echo "moving r05 $scn rc=$rc"; hard $rc; exit $rc; }
        fi
      done
      unset RTAMD_DEBUG_KNOBS
      python3 tools/moving_summary.py $OUT/moving.jsonl ;;
    asm)
      # multi-device frame assembly, host-side (default) against device-side (RT_ASM_DEVICE), 2 and 8 replicas of
      # the scene on the box's one GPU; interleaved reps
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2; do
        for d in 0,0 0,0,0,0,0,0,0,0; do
          n=$(echo $d | tr ',' ' ' | wc -w)
          for h in 0 1; do
            RT_ASM_DEVICE=$h timeout -k 10 300 python bench.py --gpus $n --devices $d --steps 20 --warmup 5 --no-cpu --no-extra \
                > $OUT/asm_${n}_h${h}_r$rep.json 2> $OUT/asm_${n}_h${h}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "asm $n h$h rc=$rc"; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/asm_${n}_h${h}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('asm n$n device$h r$rep', d['value'], d['ms_per_step'], c.get('e2e_frame_ms'), c.get('assembly_ms'), d.get('parity',{}).get('face_t_digest_equal'))"
          done
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    slotq)
      # frame-slot streams on dedicated hardware queues (default) vs the runtime's pool (RT_SLOT_POOL=1): 2 and 4
      # torchrun ranks sharing the box's GPU (gloo timing reductions), and the single-process C3 / C5 lines
      export RTAMD_DEBUG_KNOBS=1
      for rep in ${SLOTQ_REPS:-1 2}; do
        for pool in ${SLOTQ_POOLS:-0 1}; do
          for n in 2 4; do
            RT_HWQ_GPU_CAP=${HWQCAP:-8} RT_SLOT_POOL=$pool BENCH_DEVICE=0 BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
                --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n + 10 * pool)) bench.py --gpus $n \
                --steps 20 --warmup 5 --no-cpu --no-e2e > $OUT/slotq_n${n}_p${pool}_r$rep.json 2> $OUT/slotq_n${n}_p${pool}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "slotq n$n pool$pool rc=$rc"; tail -5 $OUT/slotq_n${n}_p${pool}_r$rep.err; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/slotq_n${n}_p${pool}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('slotq n$n pool$pool r$rep', d['value'], d['ms_per_step'], [p['kernel_ms_per_frame'] for p in c['per_gpu']])"
          done
          for sc in soup:primary bunny:full; do
            IFS=: read scn md <<< "$sc"
            RT_SLOT_POOL=$pool timeout -k 10 120 python bench.py --scene $scn --mode $md --steps 20 --warmup 5 --no-cpu --no-side \
                --no-extra --no-e2e --no-stats --no-cold --no-moving > $OUT/slotq_1_${scn}_p${pool}_r$rep.json 2> $OUT/slotq_1_${scn}_p${pool}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "slotq 1 $scn rc=$rc"; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/slotq_1_${scn}_p${pool}_r$rep.json').read().strip().splitlines()[-1]);print('slotq 1proc $scn pool$pool r$rep', d['value'], d['ms_per_step'])"
          done
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    rehearse8)
      # the driver's 8-GPU launch rehearsed on the box's one GPU: torchrun 8 ranks (gloo timing reductions), the
      # scene built once by rank 0 and loaded by the others, cold + prewarmed C4 shards, e2e frame over gloo
      BENCH_DEVICE=0 BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
          --master-addr 127.0.0.1 --master-port 29788 bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu \
          > $OUT/rehearse8.json 2> $OUT/rehearse8.err
      rc=$?; echo "rehearse8 rc=$rc"; cat $OUT/rehearse8.json; hard $rc ;;
    cli)
      # the drop-in CLI (host/main.cpp) on the C3 scene: scene setup time with the library default builders
      timeout -k 10 300 python tools/cli_c3.py > $OUT/cli_c3.json 2> $OUT/cli_c3.err
      rc=$?; echo "cli rc=$rc"; cat $OUT/cli_c3.json; hard $rc ;;
    c2diag)
      # C2 (bunny PRIMARY, 4 frames in flight) run to run: the library as built, the round-5 per-process queue cap
      # (RT_HWQ_GPU_CAP=1000), every slot on the pool (RT_SLOT_POOL=1); fresh process each
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2 3; do
        for v in ${C2V:-lib cap1000 pool}; do
          case $v in lib) envs="";; cap1000) envs="RT_HWQ_GPU_CAP=1000";; pool) envs="RT_SLOT_POOL=1";;
                     ss) envs="RT_SYNC_STREAMS=1";; sb) envs="RT_SORT_BEFORE=1";; both) envs="RT_SYNC_STREAMS=1 RT_SORT_BEFORE=1";;
                     r06a) envs="RTAMD_LIB=$PWD/ray-tracing-project_amd/lib/librtamd_r06a.so";; esac
          env $envs timeout -k 10 120 python bench.py --scene bunny --mode primary --steps 40 --warmup 5 --no-cpu --no-side \
              --no-extra --no-e2e --no-stats --no-cold --no-moving > $OUT/c2diag_${v}_r$rep.json 2> $OUT/c2diag_${v}_r$rep.err
          rc=$?; [ $rc -ne 0 ] && { echo "c2diag $v rc=$rc"; hard $rc; exit $rc; }
          python3 -c "import json;d=json.loads(open('$OUT/c2diag_${v}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('c2diag $v r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], c['kernel_ms_per_frame'])"
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    hybrid)
      # the counting run's packet -> per-lane hybrid model (C3 soup, C2 bunny)
      timeout -k 10 300 python tools/hybrid_model.py soup bunny > $OUT/hybrid_model.jsonl 2> $OUT/hybrid_model.err
      rc=$?; echo "hybrid rc=$rc"; cat $OUT/hybrid_model.jsonl; hard $rc ;;
    c5waves)
      # FULL megakernel occupancy A/B (small-scene build 5 / 6 / 7 waves per SIMD), C5 in flight and alone
      TAG=$TAG/c5waves LIBS="default w5 w7" CFGS="bunny:full:4 bunny:full:1" REPS=3 STEPS=50 timeout -k 10 900 \
          bash tools/ablibs.sh > $OUT/c5waves.txt 2>&1
      rc=$?; echo "c5waves rc=$rc"; cat $OUT/c5waves.txt; hard $rc ;;
    queues)
      # frames in flight vs hardware-queue assignment (tools/queue_probe.py), a fresh process per line
      for sc in bunny soup; do
        for v in ${QVARIANTS:-plain pre1 pre2 pre3 second keep2}; do
          for f in 1 4; do
            timeout -k 10 120 python tools/queue_probe.py $v $sc $f >> $OUT/queues.jsonl 2>> $OUT/queues.err
            rc=$?; [ $rc -ne 0 ] && { echo "queue probe $v $sc $f rc=$rc"; hard $rc; exit $rc; }
          done
        done
        GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/queue_probe.py plain $sc 4 >> $OUT/queues.jsonl 2>> $OUT/queues.err
        rc=$?; [ $rc -ne 0 ] && { echo "queue probe hwq8 rc=$rc"; hard $rc; exit $rc; }
      done
      cat $OUT/queues.jsonl ;;
    c3split)
      # lone C3 frames: the costliest waves as 16-lane sub-waves also for a large scene (RT_SPLIT_KP_ANY), K waves
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2; do
        for k in none 256 512 1024 2048; do
          if [ $k = none ]; then envs=""; else envs="RT_SPLIT_KP_ANY=1 RT_SPLIT_KP=$k"; fi
          env $envs timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-side --no-extra --no-e2e \
              --frames-in-flight 1 > $OUT/c3split_${k}_r$rep.json 2> $OUT/c3split_${k}_r$rep.err
          rc=$?; [ $rc -ne 0 ] && { echo "c3split $k rc=$rc"; hard $rc; exit $rc; }
          python3 -c "import json;d=json.loads(open('$OUT/c3split_${k}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('c3split $k r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'], d['roofline']['frac'], d['parity']['face_t_digest_equal'] if d.get('parity') else None)"
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    tail)
      # lone-frame tails with the product's split (tools/tail_probe.py) and the hybrid model over the FULL phases
      export RTAMD_DEBUG_KNOBS=1
      for c in c5 c3 c2; do
        RT_TIMELINE_SPLIT=1 timeout -k 10 180 python tools/tail_probe.py $c static moving >> $OUT/tail.jsonl 2>> $OUT/tail.err
        rc=$?; [ $rc -ne 0 ] && { echo "tail $c rc=$rc"; tail -5 $OUT/tail.err; hard $rc; exit $rc; }
      done
      unset RTAMD_DEBUG_KNOBS
      timeout -k 10 300 python tools/hybrid_model.py bunny:full soup:full > $OUT/hybrid_full.jsonl 2> $OUT/hybrid_full.err
      rc=$?; echo "hybrid full rc=$rc"; hard $rc
      cat $OUT/tail.jsonl $OUT/hybrid_full.jsonl ;;
    multi8)
      # eight replicas of the scene sharing the box's GPU: the in-process 8-device path end to end (enqueue workers,
      # assembly); the rate is one GPU's, the line shows the host enqueue cost per frame and per-device figures
      timeout -k 10 300 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 20 --warmup 5 --no-cpu \
          > $OUT/bench_multi8.json 2> $OUT/bench_multi8.err
      rc=$?; echo "multi8 rc=$rc"; cat $OUT/bench_multi8.json; hard $rc ;;
    fifsweep)
      # frames in flight 1-4 on the bench's own 20-step lines (C3 headline; C5 as the bench's workload), interleaved reps
      for rep in 1 2; do
        for sc in soup bunny; do
          md=primary; [ $sc = bunny ] && md=full
          for f in 1 2 3 4; do
            timeout -k 10 120 python bench.py --scene $sc --mode $md --steps 20 --warmup 5 --no-cpu --no-side --no-extra \
                --no-e2e --no-stats --frames-in-flight $f > $OUT/fif_${sc}_${f}_r$rep.json 2> $OUT/fif_${sc}_${f}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "fif $sc $f rc=$rc"; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/fif_${sc}_${f}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('fif $sc f$f r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'], c['kernel_ms_one_frame_alone'])"
          done
        done
      done ;;
    xcdrun)
      # run length of the chunked XCD dispatch order (RT_XCD_RUN; product 64), C3 at 4 frames in flight and alone
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2; do
        for c in 64 32 128 256; do
          for f in 4 1; do
            RT_XCD_RUN=$c timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-side --no-extra --no-e2e \
                --no-stats --frames-in-flight $f > $OUT/xcd_${c}_f${f}_r$rep.json 2> $OUT/xcd_${c}_f${f}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "xcd $c rc=$rc"; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/xcd_${c}_f${f}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('xcd $c f$f r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'])"
          done
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    c5split)
      # lone C5 frames: the K costliest waves of the longest-first order as four 16-lane sub-waves (RT_SPLIT_K; product 2048)
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2; do
        for k in ${C5K:-2048 1024 1536 3072}; do
          RT_SPLIT_K=$k timeout -k 10 120 python bench.py --scene bunny --mode full --steps 40 --warmup 5 --no-cpu --no-side \
              --no-extra --no-e2e --no-stats --frames-in-flight 1 > $OUT/c5split_${k}_r$rep.json 2> $OUT/c5split_${k}_r$rep.err
          rc=$?; [ $rc -ne 0 ] && { echo "c5split $k rc=$rc"; hard $rc; exit $rc; }
          python3 -c "import json;d=json.loads(open('$OUT/c5split_${k}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('c5split $k r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'])"
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    c5knob)
      # lone C5 frames under one debug knob: KNOB=<env name> VALS="<values>" (first value = the product's)
      export RTAMD_DEBUG_KNOBS=1
      for rep in 1 2; do
        for v in $VALS; do
          env $KNOB=$v timeout -k 10 120 python bench.py --scene bunny --mode full --steps 40 --warmup 5 --no-cpu --no-side \
              --no-extra --no-e2e --no-stats --frames-in-flight ${FIF:-1} > $OUT/c5knob_${KNOB}_${v}_r$rep.json 2> $OUT/c5knob_${KNOB}_${v}_r$rep.err
          rc=$?; [ $rc -ne 0 ] && { echo "c5knob $KNOB=$v rc=$rc"; hard $rc; exit $rc; }
          python3 -c "import json;d=json.loads(open('$OUT/c5knob_${KNOB}_${v}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('c5knob $KNOB=$v r$rep', d['value'], d['ms_per_step'], c['kernel_ms_one_frame_alone'])"
        done
      done
      unset RTAMD_DEBUG_KNOBS ;;
    steps)
      # the timed-step count's effect on the C3 line (20 = the driver's), 4 frames in flight
      for rep in 1 2; do
        for k in 20 40 100; do
          timeout -k 10 120 python bench.py --steps $k --warmup 5 --no-cpu --no-side --no-extra --no-e2e --no-stats \
              > $OUT/steps_${k}_r$rep.json 2> $OUT/steps_${k}_r$rep.err
          rc=$?; [ $rc -ne 0 ] && { echo "steps $k rc=$rc"; hard $rc; exit $rc; }
          python3 -c "import json;d=json.loads(open('$OUT/steps_${k}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('steps $k r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'])"
        done
      done ;;
    prewarm)
      # GPU state at the timed region's start: frames rendered back to back for P ms before the 5 warmup steps (C3)
      for rep in 1 2; do
        for pw in 0 30 100 300; do
          for k in 20 100; do
            timeout -k 10 120 python bench.py --steps $k --warmup 5 --prewarm-ms $pw --no-cpu --no-side --no-extra --no-e2e \
                --no-stats > $OUT/pw_${pw}_${k}_r$rep.json 2> $OUT/pw_${pw}_${k}_r$rep.err
            rc=$?; [ $rc -ne 0 ] && { echo "prewarm $pw rc=$rc"; hard $rc; exit $rc; }
            python3 -c "import json;d=json.loads(open('$OUT/pw_${pw}_${k}_r$rep.json').read().strip().splitlines()[-1]);c=d['config'];print('prewarm $pw steps $k r$rep', d['value'], d['ms_per_step'], c['kernel_ms_per_frame'])"
          done
        done
      done ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    multi)
      # the in-process multi-device path (no launcher) with two replicas sharing the box's GPU
      timeout -k 10 300 python bench.py --gpus 2 --devices 0,0 --steps 20 --warmup 5 > $OUT/bench_multi.json 2> $OUT/bench_multi.err
      rc=$?; echo "multi rc=$rc"; cat $OUT/bench_multi.json; hard $rc ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; hard $rc; [ $rc -ne 0 ] && exit $rc ;;
    ploc)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --builder ploc --no-cpu --no-side > $OUT/bench_ploc.json 2> $OUT/bench_ploc.err
      rc=$?; echo "ploc rc=$rc"; cat $OUT/bench_ploc.json; hard $rc ;;
    profc2)
      OUTDIR=$OUT/profc2 \
      BENCH_ARGS="--scene bunny --mode primary --steps 20 --warmup 3 --no-cpu --no-extra --no-e2e --no-side --frames-in-flight 1" \
      PMC_ARGS="--scene bunny --mode primary --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --no-side --frames-in-flight 1" \
      bash tools/profile.sh > $OUT/profile_c2.log 2>&1
      rc=$?; echo "profile c2 rc=$rc"; tail -12 $OUT/profile_c2.log; hard $rc ;;
    plocsweep)
      # PLOC A/B: neighbour radius x collapse node cost x leaf rule (C3, --builder ploc), then the SBVH line
      export RTAMD_DEBUG_KNOBS=1
      for cfg in 24:0.7:0 32:0.7:0 16:0.7:0 24:0.5:0 24:1.0:0 24:0.7:1 32:0.5:1 24:1.0:1; do
        IFS=: read r tr ru <<< "$cfg"
        RT_PLOC_RADIUS=$r RT_PLOC_TRAV=$tr RT_PLOC_RULE=$ru timeout -k 10 120 python bench.py --steps 20 --warmup 5 \
            --builder ploc --no-cpu --no-side --no-extra > $OUT/ploc_$cfg.json 2> $OUT/ploc_$cfg.err
        rc=$?; echo "ploc $cfg rc=$rc $(python3 tools/ploc_line.py $OUT/ploc_$cfg.json)"; hard $rc
      done ;;
    builders)
      # the same C3 line per builder (SBVH default, host binned SAH, device LBVH) and PLOC radii
      export RTAMD_DEBUG_KNOBS=1
      for cfg in ${BUILDERS:-sbvh sah sahgpu sbvhgpu lbvh ploc:4}; do
        IFS=: read b r <<< "$cfg"
        RT_PLOC_RADIUS=${r:-24} timeout -k 10 120 python bench.py --steps 20 --warmup 5 --builder $b --no-cpu --no-side \
            --no-extra > $OUT/builder_$cfg.json 2> $OUT/builder_$cfg.err
        rc=$?; echo "builder $cfg rc=$rc $(python3 tools/ploc_line.py $OUT/builder_$cfg.json)"; hard $rc
      done ;;
    prof)
      OUTDIR=$OUT/prof bash tools/profile.sh > $OUT/profile.log 2>&1
      rc=$?; echo "profile rc=$rc"; tail -12 $OUT/profile.log; hard $rc ;;
    profc5)
      OUTDIR=$OUT/profc5 \
      BENCH_ARGS="--scene bunny --mode full --steps 20 --warmup 3 --no-cpu --no-extra --no-e2e --no-side --frames-in-flight 1" \
      PMC_ARGS="--scene bunny --mode full --steps 5 --warmup 1 --no-cpu --no-stats --no-extra --no-e2e --no-side --frames-in-flight 1" \
      bash tools/profile.sh > $OUT/profile_c5.log 2>&1
      rc=$?; echo "profile c5 rc=$rc"; tail -12 $OUT/profile_c5.log; hard $rc ;;
  esac
done
exit 0
