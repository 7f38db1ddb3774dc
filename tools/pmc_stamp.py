#!/usr/bin/env python3
"""Record in PMC summaries (tools/pmc_summary.py, tools/pmc_traffic.py output) the library
they were measured on: pmc_stamp.py SHA16 FILE.json...  bench.py quotes the counts with
`valu_source_matches_library` = whether its own libr0hip.so has that fingerprint."""
import json
import sys


def main(sha, paths):
    for p in paths:
        with open(p) as f:
            d = json.load(f)
        d["lib_sha256_16"] = sha
        with open(p, "w") as f:
            json.dump(d, f)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
