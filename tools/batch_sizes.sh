#!/bin/bash
# tools/batch_sizes.sh [N...] -- per-kernel times of the round trip at several
# batch sizes (does the Infinity Cache keep a batch's rows between the
# remainder and the apply?), one bench.py run per size, each under its own
# time limit.  Output: gpurun_out/bsz_N.json (the bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
F="--no-c4 --no-cpu-baseline --no-host --no-latency --no-mixed --no-erasure"
sizes=${*:-1048576 524288 262144}
for b in $sizes; do
    timeout -k 10 200 python bench.py --batch "$b" $F > "gpurun_out/bsz_$b.json" 2> "gpurun_out/bsz_$b.err" || exit 3
    echo "batch $b done"
done
