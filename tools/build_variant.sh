#!/bin/bash
# Compile-time A/B: build the extension with a source patch applied, keep it as
# tensorflow_k8s_amd/_C_<name>.so, restore the sources and rebuild the baseline. Load the variant with
# TFK_C_PATH=tensorflow_k8s_amd/_C_<name>.so (ops/_lib.py).   bash tools/build_variant.sh <name> <patch>
set -e
NAME=$1; PATCH=$2
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
git apply "$PATCH"
trap 'git apply -R "$PATCH"' EXIT
python tools/build_ext.py
cp tensorflow_k8s_amd/_C.cpython-310-x86_64-linux-gnu.so "tensorflow_k8s_amd/_C_${NAME}.so"
git apply -R "$PATCH"
trap - EXIT
python tools/build_ext.py
echo "variant: tensorflow_k8s_amd/_C_${NAME}.so"
