#!/bin/bash
# Register / scratch / occupancy per kernel of a .hip file: tools/kres.sh <file.hip> [name-regex] [extra hipcc flags]
f=$1; pat=${2:-.}; shift; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics --offload-arch=gfx950 "$@" -c "$f" \
    -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 "$(dirname "$0")/kres.py" "$pat"
