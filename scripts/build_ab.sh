#!/usr/bin/env bash
# Builds the product library as of git revision REV (default HEAD) into
# level-ip_amd/ab/liblvlip_csum_ab.so, for same-process A/B runs against the
# working tree (scripts/ab.py: AB_ALT_LIB=level-ip_amd/ab/liblvlip_csum_ab.so,
# variants prefixed "alt/").  Build container only; the .so travels to the box.
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
git -C "$ROOT" archive "$REV" level-ip_amd/csrc include | tar -x -C "$T"
OUT=$ROOT/level-ip_amd/ab
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
F="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -I$T/include -fvisibility=hidden"
gcc -O2 -fPIC -fvisibility=hidden -I$T/include -c $T/level-ip_amd/csrc/csum_cpu.c -o $T/csum_cpu.o
gcc -O2 -fPIC -fvisibility=hidden -I$T/include -c $T/level-ip_amd/csrc/skb_batch.c -o $T/skb_batch.o
$HIPCC $F -c $T/level-ip_amd/csrc/csum_kernels.hip -o $T/csum_kernels.o
# revisions up to round 2 had the device frame calls in skb_dev.hip; from round 3
# the library carries a build id (build_id.c)
[ -f $T/level-ip_amd/csrc/skb_dev.hip ] && $HIPCC $F -c $T/level-ip_amd/csrc/skb_dev.hip -o $T/skb_dev.o
[ -f $T/level-ip_amd/csrc/build_id.c ] && gcc -O2 -fPIC -fvisibility=hidden -I$T/include \
    -DLVLIP_BUILD_ID="\"ab-$REV\"" -c $T/level-ip_amd/csrc/build_id.c -o $T/build_id.o
$HIPCC $F -x hip -c $T/level-ip_amd/csrc/csum_ctx.cpp -o $T/csum_ctx.o
$HIPCC -shared -fPIC --offload-arch=gfx950 -o $OUT/liblvlip_csum_ab.so $T/*.o \
    -Wl,-soname,liblvlip_csum_ab.so -Wl,-Bsymbolic-functions
echo "$OUT/liblvlip_csum_ab.so ($REV)"
