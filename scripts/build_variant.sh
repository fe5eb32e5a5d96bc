#!/bin/bash
# A/B builds of the temporal-blocking kernel: copy csrc/kernels, apply a sed
# expression to jacobi5tb.hpp, rebuild its translation units and link a
# libgmt.so into build/var/NAME/ (run a binary against it with
# LD_LIBRARY_PATH=build/var/NAME: the apps' RUNPATH yields to it).
#   scripts/build_variant.sh p4 's/constexpr int kP = 6;/constexpr int kP = 4;/'
#   scripts/build_variant.sh head git:HEAD     (jacobi5tb.hpp + .hip as committed at HEAD)
#   (the rejected round-3 candidates live in git history: git show a32db55:csrc/bench/jacobi5tb_pair.hpp)
#   scripts/build_variant.sh x cur             (the working tree's kernel sources as they are)
set -e
cd "$(dirname "$0")/.."
name=$1; expr=$2
D=build/var/$name
rm -rf $D && mkdir -p $D/src $D/obj
cp csrc/kernels/*.hpp csrc/kernels/jacobi5tb*.hip $D/src/
# the strip geometry travels with the kernel (quote includes resolve next to
# jacobi5tb.hpp first): GEOM='sed expr' edits it, e.g. the wide K = 20 kernel
#   GEOM='s/kWideK20 = false/kWideK20 = true/' scripts/build_variant.sh wide git:09d882f
#   (the wide strip left the production header in round 5; with git:REV the
#   geometry header comes from REV too)
mkdir -p $D/src/gmt && cp csrc/include/gmt/tb_geom.h $D/src/gmt/
[ -n "$GEOM" ] && sed -i "$GEOM" $D/src/gmt/tb_geom.h
case "$expr" in
  git:*) git show "${expr#git:}:csrc/kernels/jacobi5tb.hpp" > $D/src/jacobi5tb.hpp
         git show "${expr#git:}:csrc/kernels/jacobi5tb.hip" > $D/src/jacobi5tb.hip
         git show "${expr#git:}:csrc/include/gmt/tb_geom.h" > $D/src/gmt/tb_geom.h
         [ -n "$GEOM" ] && sed -i "$GEOM" $D/src/gmt/tb_geom.h ;;
  file:*) cp "${expr#file:}" $D/src/jacobi5tb.hpp ;;
  cur) ;;
  *) sed -i "$expr" $D/src/jacobi5tb.hpp ;;
esac
[ "$expr" != cur ] && cmp -s csrc/kernels/jacobi5tb.hpp $D/src/jacobi5tb.hpp && { echo "sed changed nothing"; exit 1; }
[ -n "$GEOM" ] && [ "${expr#git:}" = "$expr" ] && cmp -s csrc/include/gmt/tb_geom.h $D/src/gmt/tb_geom.h && { echo "GEOM changed nothing"; exit 1; }
# ONLY=kf: rebuild only that instantiation unit (+ jacobi5tb.hip) and take
# the other K from the production build (each unit's device code is its own
# code object, so the units need not share the edited header)
srcs=$(ls $D/src/jacobi5tb*.hip)
[ -n "$ONLY" ] && srcs="$D/src/jacobi5tb_$ONLY.hip $D/src/jacobi5tb.hip"
echo $srcs | tr ' ' '\n' | xargs -P 8 -I{} sh -c '/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Icsrc/include -munsafe-fp-atomics -c {} -o '$D'/obj/$(basename {} .hip).o'
others=$(ls build/obj/kernels/*.o | grep -v jacobi5tb)
if [ -n "$ONLY" ]; then
  for o in build/obj/kernels/jacobi5tb_k*.o; do [ -e $D/obj/$(basename $o) ] || others="$others $o"; done
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libgmt.so $D/obj/*.o $others build/obj/runtime/rt_hip.o \
  -Wl,-soname,libgmt.so -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lrocprofiler-sdk-roctx -ldl
echo "built $D/libgmt.so"
