#!/bin/bash
# One line per kernel of kernels.hip: VGPRs, AGPRs, scratch bytes/lane,
# occupancy (waves/SIMD) -- the compiler's resource-usage remarks.
# usage: tools/kernel_resources.sh [extra hipcc flags]
cd "$(dirname "$0")/../netrep_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c kernels.hip -o /tmp/kr_kernels.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/^Function Name:/ {if (n) print line; line=$3; n=1; next}
       /^VGPRs:|^AGPRs:|^ScratchSize|^Occupancy/ {line=line "  " $0}
       END {if (n) print line}' | c++filt | sed 's/nr::ProfileParams//; s/nr::NetParams//'
