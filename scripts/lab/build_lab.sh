#!/bin/bash
# Build the GEMM lab executable against the in-tree libk3m_hip.so (gfx950).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -o gemm_lab gemm_lab.hip -L../../k3m_amd -lk3m_hip -Wl,-rpath,'$ORIGIN/../../k3m_amd'
