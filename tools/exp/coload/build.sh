#!/bin/bash
# Builds the coload probe (container side; the binary runs on the GPU box).
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 a.hip b.hip -o coload
