#!/bin/bash
# tools/kres.sh FILE.hip -- per-kernel VGPRs / scratch bytes per lane of a HIP source (gfx950)
f=${1:?usage: kres.sh file.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 $KRES_FLAGS -I"$(dirname "$0")/../include" \
    -I"$(dirname "$0")/../libpoporon_amd/csrc" -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
    sed -e 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
    awk '/Function Name:/{n=$NF} /VGPRs:/{v=$NF} /ScratchSize/{print n, "vgpr=" v, "scratch=" $NF}'
