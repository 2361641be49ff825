#!/bin/bash
# Build an experimental variant of the library: scripts/build_exp.sh NAME "-DFOO=1 -DBAR=2"
set -eu
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $2 -I include \
  frender_amd/csrc/fr_kernels.hip frender_amd/csrc/fr_api.hip frender_amd/csrc/fr_demux.hip frender_amd/csrc/fr_deflate.hip frender_amd/csrc/fr_gz.cpp frender_amd/csrc/fr_csv.cpp -lz -ldl -pthread -o frender_amd/libfrender_hip_exp_$1.so
