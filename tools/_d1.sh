set -e
B="python bench.py --no-cpu-baseline --no-roofline --no-k64 --no-distortion --no-dp-rehearsal --train-steps 6 --train-warmup 2"
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/d1_g_def.log 2>&1
TMAE_LIB=ab/libtmae_gbk32.so timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/d1_g_bk32.log 2>&1
timeout -k 10 120 python tools/qkv_attn_bench.py > gpurun_out/d1_qa_def.log 2>&1
TMAE_LIB=ab/libtmae_qadec32.so timeout -k 10 120 python tools/qkv_attn_bench.py > gpurun_out/d1_qa_dec32.log 2>&1
timeout -k 10 300 $B > gpurun_out/d1_b_def.log 2>&1
TMAE_LIB=ab/libtmae_gbk32.so timeout -k 10 300 $B > gpurun_out/d1_b_bk32.log 2>&1
echo done
