# Build a variant of libhiphuff.so with extra compile flags for same-box A/B
# (tools/gpu_ab.sh): bash tools/mkvar.sh NAME "-DFOO=1 ..." -> build/var/NAME.so
set -e
cd "$(dirname "$0")/.."
N=$1; shift
D=build/var/$N
mkdir -p $D
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -Wno-comment -Iinclude -Ihuffmandecoderongpus_amd/csrc $*"
/opt/rocm/bin/hipcc $F -c huffmandecoderongpus_amd/csrc/hh_device.hip -o $D/hh_device.o &
/opt/rocm/bin/hipcc $F -c huffmandecoderongpus_amd/csrc/hh_fsm.hip -o $D/hh_fsm.o &
/opt/rocm/bin/hipcc $F -c huffmandecoderongpus_amd/csrc/hh_one.hip -o $D/hh_one.o &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/var/$N.so $D/hh_device.o $D/hh_fsm.o $D/hh_one.o build/hh_huff.o build/hh_plugin.o build/hh_encode.o build/hh_probe.o
rm -rf $D
echo build/var/$N.so
