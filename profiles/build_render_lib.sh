#!/bin/bash
# profiles/build_render_lib.sh NAME "DEFINES": icon-ray-tracing_amd/libicon_rt_hip_NAME.so, the
# product library (make lib) with irt_render.hip rebuilt under extra defines (an A/B build, e.g.
# -DIRT_HELD_ARGS, -DIRT_FRESH_LATE).  Run on the CPU host after `make lib`; the library travels
# to the GPU box like the others and is loaded through IRT_LIB_PATH.
set -e
NAME=${1:?name}; DEFS=${2:?defines}
P=$(cd "$(dirname "$0")/../icon-ray-tracing_amd" && pwd)
X=$P/build-x-$NAME
mkdir -p $X
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -Wall -I$P/../include -I$P/csrc -I$P/host -D__HIP_PLATFORM_AMD__ \
  -mllvm -amdgpu-load-store-vectorizer=0 $DEFS -c $P/csrc/irt_render.hip -o $X/irt_render.o
B=$P/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/libicon_rt_hip_$NAME.so $B/irt_host.o $B/irt_scene.o \
  $B/irt_synth.o $B/irt_debug.o $B/irt_netcdf.o $B/irt_convert.o $B/irt_kernels.o $X/irt_render.o \
  $B/irt_context.o $B/irt_build.o -lpthread
