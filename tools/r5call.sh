mkdir -p gpurun_out
timeout -k 10 120 ./tools/diag/mfma_clock_shape > gpurun_out/clock_shape.log 2>&1; cat gpurun_out/clock_shape.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/split_default.log 2>&1 || { tail -30 gpurun_out/split_default.log; exit 1; }
tail -2 gpurun_out/split_default.log
ASTYLE_GRAM_BWD_PIPE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread -k "not gatys" > gpurun_out/split_pipe.log 2>&1 || { tail -30 gpurun_out/split_pipe.log; exit 1; }
tail -2 gpurun_out/split_pipe.log
bash tools/r5ab.sh "r4||" "head||" "pipe|ASTYLE_GRAM_BWD_PIPE=1|" "r4_g||--gatys" "head_g||--gatys" "r4_b||" "head_b||" "pipe_b|ASTYLE_GRAM_BWD_PIPE=1|"
ASTYLE_LIB=audio_style_transfer_amd/libastyle_memset.so timeout -k 10 300 python -u tools/determinism2.py > gpurun_out/det_memset_glc.log 2>&1; tail -8 gpurun_out/det_memset_glc.log
