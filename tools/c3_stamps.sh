#!/bin/bash
# Phase stamps of the C3-shaped n <= 32 attention launches (diagnostic build).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c3stamps}
mkdir -p $O
cd $R
SV2N_LIB=$R/spotv2net_amd/libsv2n_stamps.so timeout -k 10 120 python tools/stamps.py c3 > $O/stamps_c3.txt 2>&1 || exit 1
SV2N_LIB=$R/spotv2net_amd/libsv2n_stamps.so timeout -k 10 120 python tools/stamps.py 512 > $O/stamps_c2.txt 2>&1 || exit 2
cat $O/stamps_c3.txt $O/stamps_c2.txt | grep -v amdgpu.ids
