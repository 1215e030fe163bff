cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
NPS_FUSE_PROLOGUE=1 timeout -k 10 300 python -u bench.py --cpu-calls 0 > gpurun_out/pro_wide_bench.log 2>&1 && tail -1 gpurun_out/pro_wide_bench.log && \
NPS_FUSE_PROLOGUE=1 NPS_X3_WIDE=0 timeout -k 10 300 python -u bench.py --cpu-calls 0 > gpurun_out/pro_narrow_bench.log 2>&1 && tail -1 gpurun_out/pro_narrow_bench.log && \
NPS_FUSE_PROLOGUE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pro_prof -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-calls 0 > gpurun_out/pro_prof.log 2>&1
