#!/bin/bash
# profiles/build_probe_lib.sh: icon-ray-tracing_amd/libicon_rt_hip_probe.so, the A/B variant
# library (make VARIANTS=all) with the measurement-only probe exits compiled in
# (-DIRT_PROBE_BUILD: IRT_PROBE_EXIT 6, 7, 8..13, 16, 17; irt_render.hip).  Run on the CPU host
# after `make VARIANTS=all lib`; the library travels to the GPU box like the others.
set -e
P=$(cd "$(dirname "$0")/../icon-ray-tracing_amd" && pwd)
mkdir -p $P/build-x5
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -Wall -I$P/../include -I$P/csrc -I$P/host -D__HIP_PLATFORM_AMD__ \
  -mllvm -amdgpu-load-store-vectorizer=0 -DIRT_ALL_VARIANTS -DIRT_PROBE_BUILD -c $P/csrc/irt_render.hip -o $P/build-x5/irt_render.o
B=$P/build-all
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/libicon_rt_hip_probe.so $B/irt_host.o $B/irt_scene.o \
  $B/irt_synth.o $B/irt_debug.o $B/irt_netcdf.o $B/irt_convert.o $B/irt_kernels.o $P/build-x5/irt_render.o \
  $B/irt_context.o $B/irt_build.o -lpthread
