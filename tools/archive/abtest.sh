#!/bin/bash
# Build tools/abtest_<name>: A = xs_kernels.hip at git revision $AREF (default HEAD) or, with
# AREF=tree, the working tree; B = the working tree's xs_kernels.hip with the given -D macros.
#   usage: [AREF=<rev>|tree] tools/archive/abtest.sh <name> [-DMACRO=...]...
#   AFLAGS="-D..." adds macros to build A as well.
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
D=/tmp/abtest
mkdir -p $D
AREF=${AREF:-HEAD}
if [ "$AREF" = tree ]; then
  cp rclone_amd/csrc/xs_kernels.hip $D/a_src.hip
  cp rclone_amd/csrc/*.h $D/
else
  for h in $(git ls-tree --name-only "$AREF" rclone_amd/csrc/ | grep '\.h$'); do git show "$AREF":$h > $D/$(basename $h); done
  git show "$AREF":rclone_amd/csrc/xs_kernels.hip > $D/a_src.hip
  git show "$AREF":rclone_amd/csrc/xs_internal.h > $D/xs_internal.h
fi
mkdir -p $D/include && cp include/rclone_crypt_gpu.h $D/include/
sed -i 's#"../../include/rclone_crypt_gpu.h"#"include/rclone_crypt_gpu.h"#' $D/xs_internal.h
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $D/a_src.hip -I $D $AFLAGS -o $D/a.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c rclone_amd/csrc/xs_kernels.hip -I rclone_amd/csrc -Dxs=xs_b "$@" -o $D/b_$name.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/archive/abtest.cpp -I rclone_amd/csrc -o $D/t.o
hipcc --offload-arch=gfx950 $D/t.o $D/a.o $D/b_$name.o -o tools/abtest_$name
