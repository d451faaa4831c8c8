"""Tabulate gpurun_out/replay_ab/*.jsonl (tools/replay_ab.sh): ms per case and
implementation, and the number of distinct output digests (must be 1)."""
import collections
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/replay_ab"
rows, dig, tags = collections.defaultdict(dict), collections.defaultdict(set), []
for f in sorted(glob.glob(os.path.join(d, "*.jsonl"))):
    tag = os.path.basename(f)[:-6]
    tags.append(tag)
    for line in open(f):
        r = json.loads(line)
        k = (r["S"], r["case"])
        rows[k][tag] = r["ms"]
        dig[k].add(r["digest"])
print("%-22s" % "case" + "".join("%11s" % t for t in tags) + "  digests")
for k, v in rows.items():
    print("%-22s" % str(k) + "".join("%11.3f" % v.get(t, float("nan")) for t in tags), len(dig[k]))
