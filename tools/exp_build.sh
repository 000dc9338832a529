#!/bin/bash
# Build a generator variant of libmq.so for an A/B timing run (diagnostic, never the product):
#   tools/exp_build.sh NAME 'python statements editing the generator source in variable s
#   (and mq_api.cpp in variable api)'
# -> mythril_amd/exp/libmq_NAME.so (load it with MQ_LIB=...)
set -e
NAME="$1"; EDIT="$2"
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/mq_exp_$NAME; rm -rf $W; mkdir -p $W; cp -r $R/mythril_amd $W/; cp -r $R/include $W/
rm -rf $W/mythril_amd/exp
python3 - "$W/mythril_amd/csrc/gen_qsa.py" "$W/mythril_amd/csrc/mq_api.cpp" "$EDIT" <<'PY'
import sys
p, pa, edit = sys.argv[1], sys.argv[2], sys.argv[3]
s = open(p).read(); s0 = s
api = open(pa).read(); a0 = api
exec(edit)
assert s != s0 or api != a0, "edit changed nothing"
open(p, "w").write(s)
open(pa, "w").write(api)
PY
(cd $W && python3 -c "from mythril_amd import build; build.build()") 2>&1 | tail -2
mkdir -p $R/mythril_amd/exp; cp $W/mythril_amd/libmq.so $R/mythril_amd/exp/libmq_$NAME.so
echo built mythril_amd/exp/libmq_$NAME.so
