#!/bin/bash
# tools/variants1.sh SRC NAME "FLAGS" [NAME "FLAGS" ...] -- experiment builds that
# recompile ONE source (e.g. rs_fast.hip) with extra -D flags and link it with
# the other objects of the library build (libpoporon_amd/obj, `make` first):
# build/NAME.so.  Time them on the GPU box with tools/exp_time.py build/NAME.so ...
cd "$(dirname "$0")/.." || exit 2
src=$1
shift
mkdir -p build
others=$(ls libpoporon_amd/obj/*.o | grep -v "/$src.o")
while [ $# -ge 2 ]; do
    name=$1 flags=$2
    shift 2
    (/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Iinclude \
        -Ilibpoporon_amd/csrc $flags -c -o "build/$name.o" "libpoporon_amd/csrc/$src" &&
        /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "build/$name.so" "build/$name.o" $others &&
        rm -f "build/$name.o") &
done
wait
ls -la build/*.so
