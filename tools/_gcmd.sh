mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python tools/decoder_trace.py > gpurun_out/trace.log 2>&1; grep -v "last done\|amdgpu.ids" gpurun_out/trace.log
