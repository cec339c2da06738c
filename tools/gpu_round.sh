mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r01l.log 2>&1 || { tail -30 gpurun_out/t_r01l.log; exit 1; }
tail -1 gpurun_out/t_r01l.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r01l.json 2> gpurun_out/bench_r01l.err || { tail -20 gpurun_out/bench_r01l.err; exit 1; }
cat gpurun_out/bench_r01l.json | cut -c1-400
bash tools/profile.sh r01l
