#!/bin/bash
# Next step for the board-major doubles ("Ranked next" 1).
# Build the guarded variant in-tree on the CPU first:
#   make -C mlp-ppo-2ply-multi_amd/csrc EXTRA="-DBGX_DBL_BM=1 -DBGX_DBL_GUARD=1" \
#        BUILD=build_dblg OUT=../bgx/libbgx_dblg.so
# and run `python -m pytest tests/test_cpuwave.py` (host emulation) before this.
# On the GPU box: the default build's reply tests, then the guarded build's
# (index checks that set err bits 0x100-0x800 instead of writing; a tripped
# check is reported as "overflow flags 0x..." by bgx_reply_moves).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dblg; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_gpu_reply.py -x -q --timeout 120 --timeout-method thread > $O/t_base.log 2>&1 || { tail -30 $O/t_base.log; exit 1; }
tail -1 $O/t_base.log
BGX_LIB=$PWD/mlp-ppo-2ply-multi_amd/bgx/libbgx_dblg.so timeout -k 10 150 python -u -m pytest tests/test_gpu_reply.py -x -q --timeout 120 --timeout-method thread > $O/t_dblg.log 2>&1 || { tail -30 $O/t_dblg.log; exit 1; }
tail -1 $O/t_dblg.log
