#!/bin/bash
# Build an A/B variant of the extension into build_ab/<name>: apply a sed expression to one source,
# build, copy the package + bench.py, restore the source and rebuild the tree.
#   tools/build_variant.sh <name> <file> '<sed expression>'
set -e
cd "$(dirname "$0")/.."
name=$1; file=$2; expr=$3
cp "$file" /tmp/variant_src.bak
sed -i "$expr" "$file"
if cmp -s "$file" /tmp/variant_src.bak; then echo "sed changed nothing"; exit 1; fi
python -m tensorflow_distributed_amd._build > /tmp/variant_build.log 2>&1 || { tail -20 /tmp/variant_build.log; cp /tmp/variant_src.bak "$file"; exit 1; }
rm -rf "build_ab/$name" && mkdir -p "build_ab/$name"
cp -r tensorflow_distributed_amd "build_ab/$name/" && cp bench.py bench_resnet.py "build_ab/$name/"
rm -rf "build_ab/$name/tensorflow_distributed_amd/__pycache__"
cp /tmp/variant_src.bak "$file"
python -m tensorflow_distributed_amd._build > /tmp/variant_build.log 2>&1 || { tail -20 /tmp/variant_build.log; exit 1; }
echo "built build_ab/$name"
