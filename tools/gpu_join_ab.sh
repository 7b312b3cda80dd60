#!/bin/bash
# Same-box A/B of setup variants (libraries under variants/<name>/, "cur" = the in-tree build): the lower-triangle
# join and H phases and learn_s of the sparse RBF sets, interleaved, three repetitions.
# usage (GPU box): tools/gpu_join_ab.sh <variant>... ; writes gpurun_out/jab/
set -e
o=gpurun_out/jab; mkdir -p $o
for rep in 1 2 3; do
  for v in "$@"; do
    lib=""; [ "$v" != cur ] && lib=PLSSVM_MI_LIB=$PWD/variants/$v/libplssvm_mi355x.so
    for c in csr_rbf_1m fp22_rbf_2m; do
      env $lib PLSSVM_MI_TIMING=1 timeout -k 10 300 python -u bench.py --config $c --solve --steps 3 --warmup 1 --no-cpu > $o/${c}_${v}_r${rep}.json 2> $o/${c}_${v}_r${rep}.err
    done
  done
done
python3 - $o <<'PY'
import json, glob, sys, re, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    name = f.split("/")[-1][:-5]
    c, v = re.match(r"(.*)_(\w+)_r\d$", name).groups()
    d = json.loads(open(f).read().strip().splitlines()[-1])
    err = open(f[:-5] + ".err").read()
    g = lambda k: float(re.search(re.escape(k) + r" ([0-9.]+)", err).group(1)) if k in err else None
    res[(c, v)].append((d["learn"]["learn_s"], g("row join, lower triangle"), g("row join, lower triangle (H)")))
out = {f"{c} {v}": {"learn_s": [r[0] for r in rs], "join_s": [r[1] for r in rs], "h_s": [r[2] for r in rs]} for (c, v), rs in res.items()}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, x in out.items(): print(k, x)
PY
