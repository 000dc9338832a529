#!/bin/bash
# HIP API trace of the drop-in stream loop (tools/stream_loop.py N M K); the db is copied back
set -o pipefail
TAG="${1:?tag}"; N="${2:-1}"; M="${3:-16}"; K="${4:-300}"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/$TAG -o run -- python3 "$R/tools/stream_loop.py" $N $M $K > "$O/loop_prof.log" 2>&1 || exit 4
db=$(find /tmp/$TAG -name '*.db' | head -1); [ -n "$db" ] && cp "$db" "$O/loop.db"
grep '"median_ms"' "$O/loop_prof.log"
