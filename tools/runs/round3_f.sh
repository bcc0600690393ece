# Round-3 session, GPU call 6: SDMA copies (bgx_dma_copy_d2h) -- probe, the
# overlap trace of the host gather's data path beside fused launches, the
# host-gather GPU test.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5f; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 python tools/copy_probe.py > $OUT/copy_plain.log 2>&1 || { tail $OUT/copy_plain.log; exit 1; }
tail -1 $OUT/copy_plain.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $OUT/dist_tests.log 2>&1 || { tail -30 $OUT/dist_tests.log; exit 1; }
tail -1 $OUT/dist_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/overlap -o run --output-format csv -- python tools/overlap_probe.py > $OUT/overlap.log 2>&1 || { tail $OUT/overlap.log; exit 1; }
grep "overlap probe" $OUT/overlap.log
python tools/overlap_check.py $OUT/overlap > $OUT/overlap.json; grep -E "fused_launches|large_copies" $OUT/overlap.json
