# Test-only device harnesses (tests/native/devcheck*.hip): built in-tree for the GPU probes.
set -e
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c devcheck_vb.hip -o /tmp/devcheck_vb.o
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c ../../charon_amd/csrc/vgroup.hip -o /tmp/devcheck_vgroup.o
$H --offload-arch=gfx950 -shared -fPIC -o libhbls_devcheck_vb.so /tmp/devcheck_vb.o /tmp/devcheck_vgroup.o
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o libhbls_devcheck_fast.so devcheck.hip
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o libhbls_devcheck_std.so devcheck_std.hip
