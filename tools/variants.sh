#!/bin/bash
# tools/variants.sh NAME "FLAGS" [NAME "FLAGS" ...] -- build experiment variants
# of the library into build/NAME.so (same sources, extra -D flags); time them
# on the GPU box with tools/exp_time.py build/NAME.so ...
cd "$(dirname "$0")/.." || exit 2
mkdir -p build
while [ $# -ge 2 ]; do
    name=$1 flags=$2
    shift 2
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude -Ilibpoporon_amd/csrc \
        -DPOPORON_BUILDTIME=1 $flags -shared -o "build/$name.so" libpoporon_amd/csrc/api.cpp \
        libpoporon_amd/csrc/rs_kernels.hip libpoporon_amd/csrc/rs_correct.hip libpoporon_amd/csrc/rs_fast.hip libpoporon_amd/csrc/rs_single.hip libpoporon_amd/csrc/rs_generic.hip libpoporon_amd/csrc/bch.hip libpoporon_amd/csrc/rng.hip &
done
wait
ls -la build/*.so
