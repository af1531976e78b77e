#!/bin/bash
# build/var/lib_<name>.so: libeigsol_hip.so with ONE source recompiled under extra defines
#   tools/build_variant.sh <name> <source.hip> [-DFOO=1 ...]   (run `make` in csrc first)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/pcsc_eigenvalue_solver_project_amd/csrc
name=$1; src=$2; shift 2
mkdir -p $R/build/var
obj=$R/build/var/${name}_${src%.hip}.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C -Wall -Wno-unused-result -Wno-unused-value "$@" -x hip -c $C/$src -o $obj
objs=""
for o in $C/build/*.o; do
  if [ "$(basename $o)" = "${src%.hip}.o" ]; then objs="$objs $obj"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/build/var/lib_$name.so $objs -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo built build/var/lib_$name.so
