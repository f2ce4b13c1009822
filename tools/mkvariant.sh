#!/bin/bash
# Make an experiment patch from sed edits of the product sources and build it:
#   tools/mkvariant.sh <name> <file relative to rray_amd/csrc> '<sed script>' [<file> '<sed>' ...]
# -> tools/patches/<name>.patch and abtest/<name>/librray_amd.so (python -m rray_amd.build variant).
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
tmp=$(mktemp -d)
mkdir -p "$tmp/a/rray_amd" "$tmp/b/rray_amd"
cp -r rray_amd/csrc "$tmp/a/rray_amd/"; cp -r rray_amd/csrc "$tmp/b/rray_amd/"
while [ $# -ge 2 ]; do
  sed -i "$2" "$tmp/b/rray_amd/csrc/$1"; shift 2
done
(cd "$tmp" && diff -ru -x '*.orig' a b > "$OLDPWD/tools/patches/$name.patch") || true
rm -rf "$tmp"
test -s "tools/patches/$name.patch" || { echo "empty patch"; exit 1; }
python -c "import sys; sys.path.insert(0, '.'); from rray_amd import build; print(build.build_variant('$name', [], patch='tools/patches/$name.patch'))"
