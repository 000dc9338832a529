#!/bin/bash
# drop-in latency study: the stream loop plain and under a HIP API trace (db copied back), then the
# default bench line with its drop-in legs
set -o pipefail
TAG="${1:?tag}"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 200 python -u tools/stream_loop.py 1 16 300 > "$O/loop_1_16.json" 2>&1 || exit 2
timeout -k 10 200 python -u tools/stream_loop.py 16 100 100 > "$O/loop_16_100.json" 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/$TAG -o run -- python3 "$R/tools/stream_loop.py" 1 16 300 > "$O/loop_prof.log" 2>&1 || exit 4
db=$(find /tmp/$TAG -name '*.db' | head -1); [ -n "$db" ] && cp "$db" "$O/loop_1_16.db"
cd "$R"
timeout -k 10 900 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" || { tail -20 "$O/bench_c2.err"; exit 6; }
echo done
