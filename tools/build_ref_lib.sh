# build libgpuaoi.so of a git revision into goworld_amd/lib_<name>/ (A/B baselines)
# usage: bash tools/build_ref_lib.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d /tmp/gwrev.XXXX)
git -C "$root" archive "$rev" goworld_amd/csrc include Makefile | tar -x -C "$tmp"
make -s -C "$tmp" -j8 goworld_amd/lib/libgpuaoi.so
mkdir -p "$root/goworld_amd/lib_$name"
cp "$tmp/goworld_amd/lib/libgpuaoi.so" "$root/goworld_amd/lib_$name/"
rm -rf "$tmp"
echo "built $rev -> goworld_amd/lib_$name/libgpuaoi.so"
