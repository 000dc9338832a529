#!/bin/bash
# Build a generator variant of the library into mythril_amd/exp/NAME/libmq.so without touching the
# product library (A/B runs: MQ_LIB=mythril_amd/exp/NAME/libmq.so).  Each SED argument is a sed
# expression applied to gen_qsa.py of the copy.   tools/build_variant.sh NAME 'SED' ['SED' ...]
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME="${1:?name}"; shift
W=/tmp/mq_var_$NAME; rm -rf $W; mkdir -p $W; cp -r $R/mythril_amd $W/; cp -r $R/include $W/
rm -rf $W/mythril_amd/exp $W/mythril_amd/prof $W/mythril_amd/csrc/_obj $W/mythril_amd/libmq.so
for e in "$@"; do sed -i -e "$e" $W/mythril_amd/csrc/gen_qsa.py; done
(cd $W && python3 -c "from mythril_amd import build; build.build(force=True)") 2>&1 | tail -2
mkdir -p $R/mythril_amd/exp/$NAME; sync; cp $W/mythril_amd/libmq.so $R/mythril_amd/exp/$NAME/libmq.so; cmp $W/mythril_amd/libmq.so $R/mythril_amd/exp/$NAME/libmq.so
echo built mythril_amd/exp/$NAME/libmq.so
