#!/bin/bash
# Build tools/abtest_<name>: A = current xs_kernels.hip defaults, B = same source with the
# given -D macros.   usage: tools/abtest.sh <name> [-DMACRO=...]...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
D=/tmp/abtest
mkdir -p $D
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c rclone_amd/csrc/xs_kernels.hip -I rclone_amd/csrc -o $D/a.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c rclone_amd/csrc/xs_kernels.hip -I rclone_amd/csrc -Dxs=xs_b "$@" -o $D/b_$name.o
hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/abtest.cpp -I rclone_amd/csrc -o $D/t.o
hipcc --offload-arch=gfx950 $D/t.o $D/a.o $D/b_$name.o -o tools/abtest_$name
