# round 3 (za): nontemporal (streaming) hints on one box -- the in-tree build (abl/lib_evdt.so)
# against the value-block gathers as `nt` loads (NT_BLOCK), the accum/RGBA8 pixel stores as
# `nt` stores (NT_STORE) and both (NT_BOTH)
set -o pipefail
mkdir -p gpurun_out/r03za
bash profiles/ab_multi.sh gpurun_out/r03za/ab "c3 c4 c5" abl/lib_evdt.so abl/lib_NT_BLOCK.so abl/lib_NT_STORE.so abl/lib_NT_BOTH.so || exit 1
