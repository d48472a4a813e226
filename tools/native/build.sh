#!/bin/bash
# Build the calibration kernels of tools/ (not part of the product library).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC mfma_peak.hip -o mfma_peak.so
