#!/usr/bin/env python3
"""Summarise tools/c5_lib_time.py / tools/c3_time.py logs of an A/B session: one line per log (gpurun_out/<name>.log),
encode / decode cold and steady ms per case, and whether every build's stream digest agrees."""
import json
import sys

rows = []
for name in sys.argv[1:]:
    try:
        line = [l for l in open("gpurun_out/%s.log" % name) if l.startswith("{")][-1]
    except (OSError, IndexError):
        print(name, "missing")
        continue
    d = json.loads(line)
    cases = [k for k in d if k != "lib"]
    print(name.ljust(12), "  ".join("%s enc %.4f/%.4f dec %.4f/%.4f" % (c, d[c]["enc_cold"], d[c]["enc_steady"],
                                                                        d[c]["dec_cold"], d[c]["dec_steady"])
                                    for c in cases))
    rows.append(tuple(d[c].get("digest", d[c].get("stream_sum")) for c in cases))
print("digests agree:", len(set(rows)) <= 1)
