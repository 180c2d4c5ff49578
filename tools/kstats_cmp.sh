#!/bin/bash
# print the StrongSort kernels' average times of each rocprof variant dir under $1
for d in "$1"/v*/; do
  v=$(basename $d); echo "== $v $(grep -o '"ms_per_step": [0-9.]*' $1/$v.log)"
  python - $(ls $d/*kernel_stats.csv | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    import re
    m = re.search(r'(\w+_kernel)', r['Name'])
    n = m.group(1) if m else r['Name'][:28]
    print(f"  {n:28s} avg_us {float(r['AverageNs'])/1e3:9.1f} calls {r['Calls']}")
PY
done
