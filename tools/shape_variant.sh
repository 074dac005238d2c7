#!/bin/bash
# A/B build of the conv library under other planner settings (host, no GPU): plans the bench step's shapes
# with the given environment (tile targets etc., read by conv_geom) into csrc/conv_shapes_NAME.h and builds
# gpi/libgpi_hip_NAME.so with that table (GPI_SHAPES_FILE).  Run the arm with GPI_LIB_VARIANT=NAME and the
# SAME environment, so the launches plan the shapes the variant holds.
# usage: tools/shape_variant.sh NAME "VAR=VAL ..." [extra -D flags]
set -eu
NAME=$1
ENVS=$2
XD=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
env $ENVS python3 "$R/tools/gen_conv_shapes.py" --out "$R/generative-physics-informed-pde_amd/csrc/build_$NAME.conv_shapes.h"
make -C "$R/generative-physics-informed-pde_amd/csrc" -j8 OUT=../gpi/libgpi_hip_$NAME.so BUILD=build_$NAME \
    EXTRA="-DGPI_SHAPES_FILE=\\\"build_$NAME.conv_shapes.h\\\" $XD" > /tmp/shape_variant_$NAME.log 2>&1
echo "built gpi/libgpi_hip_$NAME.so ($ENVS $XD)"
