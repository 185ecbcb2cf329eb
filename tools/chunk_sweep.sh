set -o pipefail
cd /root/repo && mkdir -p gpurun_out/s6
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/share_scaling.py C2 256 1 8 > gpurun_out/s6/share_C2_k16.log 2>&1 &&
RT_CHUNK_SPP=8 timeout -k 10 300 python3 tools/share_scaling.py C2 256 1 8 > gpurun_out/s6/share_C2_c8.log 2>&1 &&
RT_CHUNK_SPP=4 timeout -k 10 300 python3 tools/share_scaling.py C2 256 1 8 > gpurun_out/s6/share_C2_c4.log 2>&1
