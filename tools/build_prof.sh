#!/bin/bash
# Build the G profile variant (gen_qsa.py QSA_PROF=1) into mythril_amd/prof/libmq.so without
# touching the product library (load it with MQ_LIB=mythril_amd/prof/libmq.so).
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/mq_prof_build; rm -rf $W; mkdir -p $W; cp -r $R/mythril_amd $W/; cp -r $R/include $W/
rm -rf $W/mythril_amd/exp $W/mythril_amd/prof $W/mythril_amd/csrc/_obj $W/mythril_amd/libmq.so
(cd $W && QSA_PROF=1 python3 -c "from mythril_amd import build; build.build(force=True)") 2>&1 | tail -2
mkdir -p $R/mythril_amd/prof; cp $W/mythril_amd/libmq.so $R/mythril_amd/prof/libmq.so
echo built mythril_amd/prof/libmq.so
