#!/bin/bash
# profiles/resources.sh: registers, spills, scratch and LDS of every k_render instantiation of the
# product build (device-only compile of csrc/irt_render.hip with the Makefile's flags)
set -e
T=${TMPDIR:-/tmp}/irt_res
mkdir -p $T
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -I$R/include -I$R/icon-ray-tracing_amd/csrc \
  -I$R/icon-ray-tracing_amd/host -D__HIP_PLATFORM_AMD__ -mllvm -amdgpu-load-store-vectorizer=0 $@ \
  --cuda-device-only -c $R/icon-ray-tracing_amd/csrc/irt_render.hip -o $T/render.co
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/render.co \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/dev.co | grep -E "^\s+\.name:|\.sgpr_count|\.vgpr_count|spill_count|private_segment_fixed|group_segment_fixed" \
  | paste - - - - - - - | grep k_render | awk '{printf "%-48s lds %6s scratch %4s sgpr %3s sgpr_spill %4s vgpr %3s vgpr_spill %3s\n", $4, $2, $6, $8, $10, $12, $14}'
