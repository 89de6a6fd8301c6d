set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/r05a
timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-c4-ref > gpurun_out/r05a/bench_c2.json 2> gpurun_out/r05a/bench_c2.err
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05a/tl -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-c4-ref > gpurun_out/r05a/tl.log 2>&1
echo trace ok
f=$(find gpurun_out/r05a/tl -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/r05a/kernel_trace_c2_2stream.csv; rm -rf gpurun_out/r05a/tl
python3 tools/stream_timeline.py gpurun_out/r05a/kernel_trace_c2_2stream.csv > gpurun_out/r05a/timeline.txt
