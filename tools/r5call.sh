mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_precision.py -x -q --timeout 200 --timeout-method thread > gpurun_out/split_default.log 2>&1 || { tail -30 gpurun_out/split_default.log; exit 1; }
tail -2 gpurun_out/split_default.log
bash tools/r5ab.sh "base|ASTYLE_LIB=audio_style_transfer_amd/libastyle_base.so|" "cur||" "base_g|ASTYLE_LIB=audio_style_transfer_amd/libastyle_base.so|--gatys" "cur_g||--gatys" "base_b|ASTYLE_LIB=audio_style_transfer_amd/libastyle_base.so|" "cur_b||" "r4_g||--gatys" "cur_g2||--gatys"
