#!/bin/bash
# Hardware-counter passes over tools/pmc_kernels.py: one rocprofv3 run per counter group
# (SQ <= 8, TCC <= 4, GRBM <= 2 per pass), plus a kernel-trace pass for durations.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop() { echo "STOP: $1 rc=$2"; exit $2; }
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc/trace -o run -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc/trace.log 2>&1 || stop trace $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc/sq -o run -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc/sq.log 2>&1 || stop sq $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc/fetch -o run -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc/fetch.log 2>&1 || stop fetch $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc/write -o run -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc/write.log 2>&1 || stop write $?
cd $R
python tools/pmc_summary.py gpurun_out/pmc --md gpurun_out/pmc/pmc_kernels.md | head -40
echo PMC_DONE
