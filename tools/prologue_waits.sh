#!/bin/bash
# Scalar-load round trips in each conv kernel's prologue (host-side, no GPU): the number of
# "s_waitcnt lgkmcnt" / "vmcnt" waits before the first LDS-DMA (global_load_lds) of the kernel.
# usage: tools/prologue_waits.sh [object.o]
O=${1:-generative-physics-informed-pde_amd/csrc/build/conv.o}
D=$(mktemp -d)
cp "$O" "$D/k.o"
(cd "$D" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null)
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn "$D"/k.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 | awk '
/^[0-9a-f]+ <.*conv_(fwd|bwd)_kernel/ { if (name != "") print name, lg, vm; name = $2; lg = 0; vm = 0; done = 0; next }
/global_load_lds/ { done = 1 }
/s_waitcnt/ && !done { if ($0 ~ /lgkmcnt/) lg++; if ($0 ~ /vmcnt/) vm++ }
END { print name, lg, vm }' | sed -e 's/<_ZN12_GLOBAL__N_1//' -e 's/Ev13gpi_conv_desc13gpi_codec_ctxNS_8ConvGeomE>://'
rm -rf "$D"
