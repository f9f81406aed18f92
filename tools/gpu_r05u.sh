# round 5: split MTA work items (tests, then the item-size A/B against the in-run copy roof)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_multi_tensor.py \
  tests/test_optimizers.py tests/test_fp8_undo_kernels.py tests/test_amp.py tests/test_graph_capture.py \
  tests/test_distributed_optimizers.py > gpurun_out/r05u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05u_tests.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
for it in 65536 16384 65536 16384; do
  APEX_AMD_MTA_ITEM=$it timeout -k 10 300 python -u tools/mta_bench.py 2>gpurun_out/r05u_err.log \
    | sed "s/\"variant\": \"default\"/\"variant\": \"item$it\"/" >> gpurun_out/r05u_mta.jsonl || exit $?
done
cat gpurun_out/r05u_mta.jsonl
