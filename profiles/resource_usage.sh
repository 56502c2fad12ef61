#!/bin/bash
# Register / scratch / LDS use of the render kernels (compile-time, no GPU):
#   bash profiles/resource_usage.sh [filter]
cd "$(dirname "$0")/../icon-ray-tracing_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -I. -I../../include -D__HIP_PLATFORM_AMD__ -mllvm -amdgpu-load-store-vectorizer=0 -DIRT_ALL_VARIANTS \
  --cuda-device-only -c irt_render.hip -o /tmp/irt_render_dev.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //' |
  paste - - - - - | grep -E "${1:-k_render}"
