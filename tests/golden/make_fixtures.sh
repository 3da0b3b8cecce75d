#!/bin/sh
# Regenerates the committed golden fixtures of tests/golden/ (run from anywhere).
#   rng_fixtures.json  std::seed_seq / std::mt19937_64 / std::normal_distribution<double> outputs of
#                      libstdc++ (g++ -O2, no fast-math), the library the reference links.
set -eu
here=$(cd "$(dirname "$0")" && pwd)
tmp=$(mktemp -d)
g++ -std=c++17 -O2 -o "$tmp/gen" "$here/gen_rng_fixtures.cpp"
"$tmp/gen" > "$here/rng_fixtures.json"
rm -rf "$tmp"
echo "wrote $here/rng_fixtures.json"
