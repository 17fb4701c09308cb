#!/bin/bash
# A/B library builds: tools/build_variant.sh <tag> "<extra hipcc flags>" -> multilinear-map-cryptography_amd/libtns_<tag>.so
# (run on the GPU box with TNS_LIB=$PWD/multilinear-map-cryptography_amd/libtns_<tag>.so)
set -euo pipefail
cd "$(dirname "$0")/../multilinear-map-cryptography_amd"
tag=$1; extra=$2
make -s -j8 libtns_$tag.so BUILD_DIR=build_$tag OUT=libtns_$tag.so EXTRA_FLAGS="$extra"
