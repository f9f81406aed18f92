#!/bin/bash
# Hardware counters of the kernels a python tool launches: one rocprofv3 run per counter group
# (each within the per-block limits: <= 8 SQ, FETCH_SIZE alone, WRITE_SIZE alone) plus a
# kernel-trace pass, joined per (kernel, grid) by tools/pmc_summary.py.
# Usage: tools/gpu_pmc_cmd.sh <tag> <script.py> [args]   -> gpurun_out/pmc_<tag>/pmc.md
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
cd /tmp
S="$R/$1"; shift
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $S "$@" > $O/trace.log 2>&1 || stop trace $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 $S "$@" > $O/sq.log 2>&1 || stop sq $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU --output-format csv -d $O/sq2 -o run -- python3 $S "$@" > $O/sq2.log 2>&1 || stop sq2 $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $S "$@" > $O/fetch.log 2>&1 || stop fetch $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $S "$@" > $O/write.log 2>&1 || stop write $?
cd $R
python tools/pmc_summary.py $O --by-grid --filter "${PMC_FILTER:-apex_amd::}" --md $O/pmc.md > /dev/null
rm -rf $O/trace $O/sq $O/sq2 $O/fetch $O/write
echo PMC_DONE
