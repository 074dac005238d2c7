#!/bin/bash
# VGPR / SGPR / spill / LDS usage of every kernel in a built object (host-side, no GPU).
# usage: tools/kernel_resources.sh [object.o] [name filter]
O=${1:-generative-physics-informed-pde_amd/csrc/build/conv.o}
F=${2:-conv_}
D=$(mktemp -d)
cp "$O" "$D/k.o"
(cd "$D" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$D"/k.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 | \
    grep -E "^\s+\.name:|\.vgpr_count|\.sgpr_count|\.vgpr_spill_count" | \
    awk '/\.name:/ {n=$2} /\.sgpr_count/ {s=$2} /\.vgpr_count/ {v=$2} /\.vgpr_spill_count/ {print n, "vgpr", v, "sgpr", s, "spill", $2}' | \
    grep "$F" | sed -e 's/_ZN12_GLOBAL__N_1//' -e 's/Ev13gpi_conv_desc13gpi_codec_ctxNS_8ConvGeomE//'
rm -rf "$D"
