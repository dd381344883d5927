set -o pipefail
PATHS=20,21 timeout -k 10 300 python -u tools/gemm_tune.py prefill enc dec256 > gpurun_out/tune.log 2>&1 || { tail -n 20 gpurun_out/tune.log; exit 1; }
QASR_LIB=light-whisper_amd/libqasr_slp.so PATHS=20,21 timeout -k 10 300 python -u tools/gemm_tune.py prefill enc dec256 > gpurun_out/tune2.log 2>&1 || { tail -n 20 gpurun_out/tune2.log; exit 1; }
grep -v amdgpu gpurun_out/tune.log; grep -v amdgpu gpurun_out/tune2.log
