#!/bin/bash
# A/B timing build of libpsg.so: tools/ab_build.sh <name> "<extra hipcc flags>" [git-rev]
# -> build/<name>/libpsg.so (sources of the working tree, or of git-rev);
# select it with PSG_LIB_PATH.  Not the product build.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; F=$2; REV=$3
O=$R/build/$N; mkdir -p $O/src
if [ -n "$REV" ]; then
  for f in $(git -C $R ls-tree --name-only $REV parameter_server_amd/csrc/); do
    git -C $R show $REV:$f > $O/src/$(basename $f); done
  mkdir -p $O/include; git -C $R show $REV:include/psg.h > $O/include/psg.h
  SRC=$O/src; sed -i 's#"../../include/psg.h"#"../include/psg.h"#' $SRC/*.hip $SRC/*.h 2>/dev/null || true
else
  SRC=$R/parameter_server_amd/csrc
fi
for f in $SRC/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero \
    -ffp-contract=off $F -c $f -o $O/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $O/libpsg.so $O/*.o -L/opt/rocm/lib -lrccl
rm -f $O/*.o
