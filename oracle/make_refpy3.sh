#!/usr/bin/env bash
# Build-container-only recipe: make the Python-2 reference
# importable under Python 3 in a SCRATCH directory outside the repository.
# Nothing produced here is committed or shipped to the GPU box; only the golden
# vectors written by tools/gen_golden.py (data) enter tests/golden/.
set -euo pipefail
REF=${REF:-/root/reference}
OUT=${OUT:-/tmp/refpy3}
[ -d "$REF/hyperopt" ] || { echo "reference not present at $REF" >&2; exit 1; }
rm -rf "$OUT" && mkdir -p "$OUT"
cp -r "$REF/hyperopt" "$OUT/"
chmod -R u+w "$OUT"
rm -rf "$OUT/hyperopt/__pycache__"
python3 -m lib2to3 -w -n "$OUT/hyperopt" >/dev/null 2>&1
# networkx 3 returns a generator from topological_sort (pyll/base.py:654-655)
sed -i 's/    order = nx.topological_sort(G)/    order = list(nx.topological_sort(G))/' "$OUT/hyperopt/pyll/base.py"
echo "$OUT"
