#!/bin/bash
# A variant of the library for A/B runs: build_variant.sh NAME "-DFLAG ..." ->
# crispresso_amd/lib/libcrispr_nw_NAME.so (select with CRISPR_NW_LIB=libcrispr_nw_NAME.so).
set -e
cd "$(dirname "$0")/../../crispresso_amd/csrc"
make -j8 OBJDIR=/tmp/nw_variant_$1 OUT=../lib/libcrispr_nw_$1.so EXTRA="$2" >/dev/null
echo "built crispresso_amd/lib/libcrispr_nw_$1.so ($2)"
