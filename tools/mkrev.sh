# Build libhiphuff.so as of a git revision, for same-box A/B against the
# working tree (tools/gpu_ab.sh): bash tools/mkrev.sh NAME REV -> build/var/NAME.so
set -e
cd "$(dirname "$0")/.."
N=$1; REV=$2
D=build/var/$N.src
rm -rf $D; mkdir -p $D/csrc $D/include
for f in $(git ls-tree --name-only $REV huffmandecoderongpus_amd/csrc/); do git show $REV:$f > $D/csrc/$(basename $f); done
for f in $(git ls-tree --name-only $REV include/); do git show $REV:$f > $D/include/$(basename $f); done
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -Wno-comment -I$D/include -I$D/csrc"
for f in $D/csrc/*.hip; do /opt/rocm/bin/hipcc $F -c $f -o $D/$(basename $f .hip).o & done
for f in $D/csrc/*.c; do gcc -O3 -fPIC -std=gnu11 -I$D/include -I$D/csrc -c $f -o $D/$(basename $f .c).o & done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/var/$N.so $D/*.o
rm -rf $D
echo build/var/$N.so
