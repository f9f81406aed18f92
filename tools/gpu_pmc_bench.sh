#!/bin/bash
# Hardware-counter passes over a short run of bench.py (the real ResNet-50 bs-256 shapes): one
# rocprofv3 run per counter group (SQ <= 8 + GRBM <= 2, FETCH_SIZE, WRITE_SIZE) plus a
# kernel-trace pass for durations, joined per kernel by tools/pmc_summary.py.
# Usage: tools/gpu_pmc_bench.sh <tag> [bench.py args]   -> gpurun_out/pmc_<tag>/pmc.md
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
cd /tmp
B="$R/bench.py --steps 2 --warmup 2 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $B > $O/trace.log 2>&1 || stop trace $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 || stop sq $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || stop fetch $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || stop write $?
cd $R
python tools/pmc_summary.py $O --by-grid --md $O/pmc.md > /dev/null
# keep only the summary (the per-dispatch CSVs are large)
rm -rf $O/trace $O/sq $O/fetch $O/write
echo PMC_DONE
