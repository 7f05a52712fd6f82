#!/bin/bash
# usage: scripts/regs.sh FILE.hip [REGEX] -- per-kernel VGPR/AGPR/spill/occupancy of a library source
# (device-only compile with the resource-usage remarks; nothing is written into the tree)
set -u
R=$(cd "$(dirname "$0")/.." && pwd)
f=$1; pat=${2:-.}
out=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$R/include \
  --cuda-device-only -c $R/poissbox_amd/csrc/$f -o $out/k.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy" |
  sed -E 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' | paste - - - - - |
  grep -E "$pat" | sed -E 's/Function Name: //; s/ScratchSize \[bytes\/lane\]/scratch/; s/\t/ /g; s/ +/ /g'
rm -rf $out
