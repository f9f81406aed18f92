mkdir -p gpurun_out
for i in 1 2; do
for v in r03 r02; do
APEX_AMD_CONV1X1_ROUTES=$v timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/ab_${v}_${i}.log 2>&1 || exit 1
echo "$v $(tail -1 gpurun_out/ab_${v}_${i}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
