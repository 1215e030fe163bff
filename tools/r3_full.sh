# Full GPU pass: all -m gpu tests, smoke, C3 bench, rocprofv3 kernel stats of the C3 bench
export TMPDIR=/tmp
T=${1:-a}
tools/gpu_steps.sh \
 "900|gpurun_out/r3_gpu_tests_$T.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200|gpurun_out/r3_smoke_$T.log|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|gpurun_out/r3_bench_$T.json|python bench.py" \
 "300|gpurun_out/r3_prof_$T.log|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python bench.py --steps 3 --warmup 1 --cpu-calls 0"
