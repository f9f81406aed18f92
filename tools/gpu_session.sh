#!/bin/bash
# One GPU-box session (gpurun): selected steps, each under its own time limit, chained so that a
# crash / timeout / fault ends the call.  STEPS is a space-separated list of:
#   tests      pytest -m gpu (TESTS selects files; default all)
#   smoke      __graft_entry__.smoke()
#   bench      1-GPU headline bench (BENCH_ARGS appended)
#   syncbn2    2 ranks sharing the GPU, gloo, --sync-bn (fused bn_group=world over peer memory)
#   prof       rocprofv3 --kernel-trace --stats of a short bench (after the APEX_BENCH_MARK spin)
#   pyprof     rocprofv3 marker + kernel trace of examples/pyprof/lenet.py through apex.pyprof parse/prof
#   script     python $SCRIPT (comma-separated tools/ micro-benchmarks), output to gpurun_out/script_<i>.log
# Test failures (rc 1) do not stop the chain; anything >= 2 does.
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export MIOPEN_USER_DB_PATH=$R/gpurun_out/miopen_udb
export MIOPEN_CUSTOM_CACHE_DIR=$R/gpurun_out/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
stop() { echo "STOP: $1 rc=$2"; exit $2; }
for s in ${STEPS:-tests smoke bench}; do
  case $s in
  tests)
    timeout -k 10 ${TESTS_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu ${PYTEST_FLAGS--x} -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && stop pytest $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && stop smoke $rc ;;
  bench)
    timeout -k 10 400 python bench.py --steps ${BSTEPS:-20} --warmup ${BWARM:-8} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
    rc=$?; tail -3 gpurun_out/bench.log; [ $rc -ne 0 ] && stop bench $rc ;;
  syncbn2)
    APEX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --sync-bn --steps 4 --warmup 3 --batch-size 64 \
      > gpurun_out/syncbn2.log 2>&1
    rc=$?; tail -4 gpurun_out/syncbn2.log; [ $rc -ne 0 ] && stop syncbn2 $rc ;;
  prof)
    cd /tmp && APEX_BENCH_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 6 ${BENCH_ARGS} > $R/gpurun_out/prof_bench.log 2>&1
    rc=$?; cd $R; tail -3 gpurun_out/prof_bench.log; [ $rc -ne 0 ] && stop prof $rc
    # summarize on the box (the raw trace db can exceed what gpurun merges back)
    python tools/prof_summary.py gpurun_out/prof_bench/bench_results.db --after spin_kernel --steps 10 --top 60 \
      --md gpurun_out/prof_summary.md --title "${PROF_TITLE:-ResNet-50 bench kernel trace}" > /dev/null 2>&1
    head -12 gpurun_out/prof_summary.md; rm -rf gpurun_out/prof_bench ;;
  pyprof)
    # apex.pyprof end to end: roctx op markers (fwd + bwd) -> rocprofv3 -> parse -> prof
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace --output-format csv \
      -d $R/gpurun_out/pyprof_trace -o run -- python3 $R/examples/pyprof/lenet.py > $R/gpurun_out/pyprof_run.log 2>&1
    rc=$?; cd $R; tail -2 gpurun_out/pyprof_run.log; [ $rc -ne 0 ] && stop pyprof $rc
    python -m apex.pyprof.parse gpurun_out/pyprof_trace > gpurun_out/pyprof_parsed.txt && \
      python -m apex.pyprof.prof -c idx,dir,sub,layer,mod,op,kernel,params,sil,tc,flops,bytes -w 240 \
        gpurun_out/pyprof_parsed.txt > gpurun_out/pyprof_report.txt && \
      python -m apex.pyprof.prof --summary op gpurun_out/pyprof_parsed.txt > gpurun_out/pyprof_summary.txt
    rc=$?; head -20 gpurun_out/pyprof_summary.txt; rm -rf gpurun_out/pyprof_trace; [ $rc -ne 0 ] && stop pyprof_post $rc ;;
  script)
    # SCRIPT: one or more comma-separated "tool.py args" entries, logs script_<i>.log
    IFS=',' read -ra scripts <<< "$SCRIPT"; i=0
    for sc in "${scripts[@]}"; do
      timeout -k 10 ${SCRIPT_TIMEOUT:-400} python $sc > gpurun_out/script_$i.log 2>&1
      rc=$?; tail -20 gpurun_out/script_$i.log; [ $rc -ne 0 ] && stop "script $sc" $rc; i=$((i+1))
    done ;;
  esac
done
du -sh gpurun_out/miopen_udb gpurun_out/miopen_cache 2>/dev/null
echo ALL_DONE
