#!/usr/bin/env bash
# Static stats of a kernel's innermost loop: kstat.sh <src.hip> <kernel-substring> [extra hipcc flags]
# Prints VGPRs/scratch and the instruction mix of the last "Inner Loop Header" block.
set -e
SRC=$1; PAT=$2; shift 2
PKG=$(cd "$(dirname "$0")/../gpu-accel-ofdm-ls-mrc_amd" && pwd)
W=$(mktemp -d)
( cd $W && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -I$PKG/build/gen -I$PKG/csrc -I$PKG/../include \
    -c $(realpath -m $PKG/../$SRC 2>/dev/null || echo $SRC) -o k.o -save-temps -Rpass-analysis=kernel-resource-usage 2> remarks.txt )
grep -A4 "Function Name: .*$PAT" $W/remarks.txt | grep -E "VGPRs:|Scratch|Occupancy" | sed 's/.*remark: *//;s/ \[-Rpass.*\]//' | tr '\n' ' '; echo
S=$(ls $W/*gfx950*.s)
L=$(grep -n "^_Z[^ ]*$PAT[^ ]*:" $S | head -1 | cut -d: -f1)
sed -n "$L,\$p" $S | awk '/s_endpgm/{print; exit} {print}' > $W/k.s
B=$(grep -n "Inner Loop Header" $W/k.s | tail -1 | cut -d: -f1)
E=$(awk -v b=$B 'NR>b && /s_cbranch/{print NR; exit}' $W/k.s)
sed -n "${B},${E}p" $W/k.s > $W/loop.s
echo "loop instrs $(grep -c '^\s*[a-z]' $W/loop.s): valu $(grep -c '^\s*v_' $W/loop.s) pk $(grep -c 'v_pk' $W/loop.s) mov $(grep -c 'v_mov_b32_e32' $W/loop.s) dpp $(grep -c '_dpp' $W/loop.s) nop $(grep -c 's_nop' $W/loop.s) ds $(grep -c '^\s*ds_' $W/loop.s) vmem $(grep -c 'global_load\|buffer_load' $W/loop.s) waitcnt $(grep -c 's_waitcnt' $W/loop.s)"
[ -n "$KSTAT_KEEP" ] && cp $W/loop.s $KSTAT_KEEP
rm -rf $W
