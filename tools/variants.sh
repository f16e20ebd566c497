#!/bin/bash
# tools/variants.sh NAME REV "FLAGS" [NAME REV "FLAGS" ...] -- build experiment
# variants of the library into build/NAME.so: the product sources at git
# revision REV ("WORK" = the working tree), plus extra -D flags.  Time them on
# the GPU box with tools/exp_bench.py build/NAME.so ... (same box, alternated).
cd "$(dirname "$0")/.." || exit 2
mkdir -p build
SRCS="api.cpp rs_kernels.hip rs_correct.hip rs_fast.hip rs_errata.hip rs_single.hip rs_generic.hip bch.hip rng.hip"
while [ $# -ge 3 ]; do
    name=$1 rev=$2 flags=$3
    shift 3
    src=libpoporon_amd/csrc
    if [ "$rev" != "WORK" ]; then
        src=$(mktemp -d /tmp/variant_XXXX)
        git archive "$rev" libpoporon_amd/csrc include | tar -x -C "$src"
        inc="$src/include"
        src="$src/libpoporon_amd/csrc"
    else
        inc=include
    fi
    files=""
    for f in $SRCS; do files="$files $src/$f"; done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -I"$inc" -I"$src" \
        -DPOPORON_BUILDTIME=1 $flags -shared -o "build/$name.so" $files &
done
wait
ls -la build/*.so
