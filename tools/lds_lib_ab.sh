#!/bin/bash
# LDS fit kernel A/B across library builds (build_variants/*.so from tools/variant.sh) and engine
# knobs, interleaved, on one box: tools/lds_ab.py per build (shapes adversarial worst many).
#   LIBS="vcodes nocache" tools/lds_lib_ab.sh      (the tree's libplacement.so always runs as "base")
set -e
export LDS_AB_CONFIGS=${LDS_AB_CONFIGS:-'[{}, {"PE_LDS_NOSORT": "1"}]'}
for rep in 1 2; do
  timeout -k 10 200 python3 tools/lds_ab.py ${SHAPES:-adversarial worst many}
  for v in ${LIBS}; do
    PE_LIBRARY=$PWD/build_variants/$v.so timeout -k 10 200 python3 tools/lds_ab.py ${SHAPES:-adversarial worst many}
  done
done
