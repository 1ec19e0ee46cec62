#!/bin/bash
# Lab build with the split replaced by one conversion (numerically wrong; timing experiment only).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -DK3M_X6_LAB_NO_SPLIT -o gemm_lab_nosplit gemm_lab.hip -L../../k3m_amd -lk3m_hip -Wl,-rpath,'$ORIGIN/../../k3m_amd'
