#!/bin/bash
# round-6 GPU call: which tier breaks C3 parity (tests/test_gpu_c3_record.py failed once at row 2024 with the
# compact bails going straight to the full tier while routing is on): every layout against the oracle every
# row, product library and the W_DIRECT_PRE=0 build
set -o pipefail
R=$(pwd); D=$R/gpurun_out/$1; mkdir -p $D
cd /tmp && export TMPDIR=/tmp; cd $R
timeout -k 10 400 python3 -u tools/dbg_c3_tiers.py default full128 full64 cap3 capm12 > $D/product.txt 2>&1 || { tail -20 $D/product.txt; exit 1; }
cat $D/product.txt | grep -v amdgpu.ids
W=/tmp/ur3e_var_direct0; rm -rf $W; mkdir -p $W; cp -r $R/ur3e_amd $R/include $W/
timeout -k 10 600 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -disable-machine-licm -Wno-unused-result -DW_DIRECT_PRE=0 -o $W/lib.so $W/ur3e_amd/csrc/ur3e_batch.hip $W/ur3e_amd/csrc/ur3e_vecnorm.hip $W/ur3e_amd/csrc/ur3e_mjcf.cpp $W/ur3e_amd/csrc/ur3e_gather.cpp -ldl > $D/direct0_build.log 2>&1 || { tail -5 $D/direct0_build.log; exit 1; }
UR3E_LIB=$W/lib.so timeout -k 10 300 python3 -u tools/dbg_c3_tiers.py default default > $D/direct0.txt 2>&1 || { tail -20 $D/direct0.txt; exit 1; }
cat $D/direct0.txt | grep -v amdgpu.ids
