#!/bin/bash
# Per-launch kernel times of one config's last step under different environment settings.
# usage: tools/gpu_kt_sweep.sh TAG CONFIG "VAR=a VAR2=b" "VAR=c" ...   ("-" = no setting)
set -o pipefail
TAG="${1:?tag}"; CFG="${2:?config}"; shift 2
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for envs in "$@"; do
  i=$((i+1))
  [ "$envs" = "-" ] && envs=""
  rm -rf /tmp/kt
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt -o run -- python3 "$R/bench.py" --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/kt_$i.json" 2> "$OUT/kt_$i.err" || { tail -20 "$OUT/kt_$i.err"; exit 5; }
  db=$(find /tmp/kt -name '*.db' | head -1); python3 "$R/tools/rocpd_summary.py" "$OUT/kt_${CFG}_$i.json" "kt=$db" > /dev/null
  python3 - "$OUT/kt_${CFG}_$i.json" "$OUT/kt_$i.json" "[$envs]" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ld = d["last_dispatches"]
i = max(k for k, x in enumerate(ld) if x["kernel"] == "mq::qs_init_best")
print(sys.argv[3], round(b["ms_per_step"], 3), b.get("parity_ok"),
      " ".join(f"{x['kernel'].split('mq::')[-1][:6]}:{x['ns']/1e3:.0f}" for x in ld[i:] if "mq::" in x["kernel"]))
PY
done
rm -rf /tmp/kt
