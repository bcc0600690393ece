#!/bin/bash
# The board-major doubles reply launch (BGX_REPLY_DBL=1), guarded: every global
# write of the movegen kernels and the reply launch's input reads check their
# index and set an error bit (0x100..0x8000) instead of touching memory out of
# range (BGX_DBL_GUARD=1; a tripped check comes back from bgx_reply_moves as
# "overflow flags 0x..."). Built in-tree on the CPU:
#   make -C mlp-ppo-2ply-multi_amd/csrc EXTRA="-DBGX_DBL_GUARD=1" BUILD=build_g OUT=../bgx/libbgx_guard.so
# Runs the reply launch test on the guarded build, per-roll doubles first (the
# guards themselves must not trip), then board-major. Run as the last step of a
# GPU call: nothing follows it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/dblg; mkdir -p $O
B=$PWD/mlp-ppo-2ply-multi_amd/bgx
for dbl in 0 1; do
  T="tests/test_gpu_reply.py::test_reply_moves_vs_oracle[1-0-$dbl-4]"
  BGX_LIB=$B/libbgx_guard.so timeout -k 10 150 python -u -m pytest "$T" -x -q --timeout 120 --timeout-method thread > $O/t_dbl$dbl.log 2>&1 || { tail -30 $O/t_dbl$dbl.log; exit 1; }
  tail -1 $O/t_dbl$dbl.log
done
