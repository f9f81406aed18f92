# round 5: MTA A/B — fast-math (default) vs IEEE variant vs ILP2 variant, each with its own copy roof
mkdir -p gpurun_out
for v in default _C_ieee.so _C_ilp2.so default; do
  if [ $v = default ]; then E=""; else E="APEX_AMD_NATIVE_SO=rocm-apex_amd/_variants/$v"; fi
  env $E timeout -k 10 300 python -u tools/mta_bench.py >> gpurun_out/r05r_mta.jsonl 2>gpurun_out/r05r_err.log || exit $?
done
cat gpurun_out/r05r_mta.jsonl
