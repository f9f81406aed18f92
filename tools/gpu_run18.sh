#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_peer_memory.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_peer.log | head -20; tail -2 gpurun_out/pytest_peer.log; [ $rc -ne 0 ] && stop pytest_peer $rc
echo ALL_DONE
