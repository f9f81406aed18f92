# round 5: fast-math optimizer kernels (tests + in-run copy roof), then the K=512 column-tile A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_optimizers.py \
  tests/test_fp8_undo_kernels.py tests/test_amp.py tests/test_conv1x1_bn.py tests/test_bottleneck_block.py \
  > gpurun_out/r05q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05q_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/mta_bench.py > gpurun_out/r05q_mta.jsonl 2>&1 || exit $?
cat gpurun_out/r05q_mta.jsonl
bash tools/ab_bench.sh r05q_nc128 "APEX_AMD_C1BN_NC128_MAXK=512" "APEX_AMD_C1BN_NC128_MAXK=256" 2
