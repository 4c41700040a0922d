#!/bin/bash
# A/B build of the mesh-kernel translation unit only: lib/variants/NAME.so = the product objects with
# csrc/kernels/render_mesh_f64.hip recompiled under EXTRA flags (e.g. -DRT_ROLES_WALKERS=5).
# Usage (from the repo root): bash tools/mesh_variant.sh NAME "-DFLAG=V ..." [TU basename, default render_mesh_f64]
set -e
NAME=$1; FLAGS=$2; TU=${3:-render_mesh_f64}
cd "$(dirname "$0")/../raytracer-server_amd"
make -s -j8 >/dev/null
rm -rf "build_$NAME"; cp -rp build "build_$NAME"
rm -f "build_$NAME/kernels/$TU.o"
make -s -j8 BUILD="build_$NAME" LIB="lib/variants/$NAME.so" EXTRA="$FLAGS" 2>&1 | grep -E "error" || true
ls -la "lib/variants/$NAME.so"
