#!/bin/bash
# WRITE_SIZE / FETCH_SIZE passes (one counter block per run) for library variants (diagnostic).
# Usage: tools/pmc_write.sh <outdir> <variant>...   (variant "main" = the in-tree library)
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  LIBV=$PWD/marl-soccer_amd/lib/variants/lib_$V.so
  [ "$V" = main ] && LIBV=$PWD/marl-soccer_amd/lib/libmarlsoccer.so
  for C in WRITE_SIZE FETCH_SIZE; do
    MARL_SOCCER_LIB=$LIBV timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/${V}_$C -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/${V}_$C.log 2>&1
    rc=$?
    echo "$V $C rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $OUT/${V}_$C.log; exit $rc; }
  done
done
exit 0
