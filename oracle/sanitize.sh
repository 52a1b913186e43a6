#!/bin/bash
# ASan + UBSan build of the CPU oracle (test infrastructure; host code only, no GPU): the oracle's CPU test suite
# run against a sanitizer build of oracle/rx_oracle.cpp. Usage: bash oracle/sanitize.sh  (from the repo root)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=/tmp/rx_oracle_san
mkdir -p $OUT
g++ -O1 -g -std=c++17 -ffp-contract=off -fopenmp -fPIC -shared -fsanitize=address,undefined -fno-omit-frame-pointer \
    -fno-sanitize-recover=undefined "$HERE/rx_oracle.cpp" -o $OUT/liboracle.so
export RX_ORACLE_LIB=$OUT/liboracle.so
export LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
export OMP_NUM_THREADS=4
python -m pytest "$HERE/../tests" -q -m "not gpu" -p no:cacheprovider -x
