#!/bin/bash
# round-6 GPU call: the C3 pick window by window on the product (mid tier 16/64 + grasp tier 24/96, list tiers
# reading their arguments through the kernarg pointer), then same-box A/B against the tier chains without the
# mid tier (mid0: round 5's; mid0g18: A/B 1's grasp 18/72) and against by-value list-tier arguments (klist0)
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 300 python3 tools/mesh_c3.py 4096 main_mesh > $D/c3_windows.jsonl 2> $D/c3_windows.err || { tail -5 $D/c3_windows.err; exit 1; }
cut -c1-230 $D/c3_windows.jsonl
AB_EXTRA=1 timeout -k 10 900 bash tools/ab_multi.sh ${ROUNDS:-2} mid0 mid0g18 klist0 2>&1 | tee $D/ab.txt
cp -r gpurun_out/ab $D/ab_raw 2>/dev/null; true
