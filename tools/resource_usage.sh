#!/bin/bash
# VGPRs / scratch / occupancy of the D=10 forward (or backward: SRC=dfwfm_train.hip) kernels, device-only compile.
cd "$(dirname "$0")/../xsdeepfwfm_deprecated_amd/csrc"
SRC=${SRC:-dfwfm_kernels.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDFWFM_KD=${KD:-10} ${EXTRA:-} -c --offload-device-only -o /tmp/ru.o $SRC \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|Scratch|Occupancy" | \
  paste - - - - | sed -E 's/[a-z_.]+:[0-9]+:[0-9]+: remark: *//g; s/\[-Rpass-analysis=kernel-resource-usage\]//g' | \
  grep -E "${FILTER:-fwd_kernelILi10ELi3ELi1ELb0ELi0ELi8|fwd_kernelILi10ELi1ELi1ELb0ELi0ELi4|fwd_kernelILi10ELi3ELi1ELb1ELi0ELi8}"
