#!/usr/bin/env python3
"""Generate tests/golden/bessd_classes.json from the reference's module
sources: per class the ADD_MODULE name template and help text
(core/module.h:731), the gate counts (kNumIGates / kNumOGates, default 1,
MAX_GATES = 8192) and the commands table (name, argument type, thread
safety) -- the data tests/test_bessd_wrappers.py holds the plugin wrappers
to. Run in the build container, where /root/reference exists:

    python scripts/gen_bessd_classes_fixture.py /root/reference
"""
import json
import os
import re
import sys

MODULES = {  # class -> reference file stem (core/modules/<stem>.{h,cc})
    "ExactMatch": "exact_match", "WildcardMatch": "wildcard_match",
    "IPChecksum": "ip_checksum", "L4Checksum": "l4_checksum",
    "HashLB": "hash_lb", "ACL": "acl", "IPLookup": "ip_lookup",
    "UpdateTTL": "update_ttl", "StaticNAT": "static_nat", "NAT": "nat",
    "IPEncap": "ip_encap", "Rewrite": "rewrite",
}


def gates(text, which):
    m = re.search(r"k%s\s*=\s*(\w+)\s*;" % which, text)
    if not m:
        return 1
    v = m.group(1)
    return 8192 if v == "MAX_GATES" else int(v)


def cmds(text, cls):
    m = re.search(r"const Commands %s::cmds\s*=\s*\{(.*?)\};" % cls, text, re.S)
    if not m:
        return []
    out = []
    for e in re.finditer(r'\{\s*"([^"]+)"\s*,\s*"([^"]+)"\s*,.*?Command::(THREAD_\w+)\s*\}',
                         m.group(1), re.S):
        out.append([e.group(1), e.group(2), e.group(3)])
    return out


def add_module(text, cls):
    m = re.search(r"ADD_MODULE\(\s*%s\s*,\s*((?:\"[^\"]*\"\s*)+),\s*((?:\"[^\"]*\"\s*)+)\)"
                  % cls, text, re.S)
    join = lambda s: "".join(re.findall(r'"([^"]*)"', s))
    return join(m.group(1)), join(m.group(2))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {}
    for cls, stem in sorted(MODULES.items()):
        base = os.path.join(ref, "core", "modules", stem)
        cc = open(base + ".cc").read()
        h = open(base + ".h").read()
        tmpl, help_ = add_module(cc, cls)
        out[cls] = {"name_template": tmpl, "help": help_,
                    "igates": gates(h, "NumIGates"), "ogates": gates(h, "NumOGates"),
                    "cmds": cmds(cc, cls)}
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "tests", "golden", "bessd_classes.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(dst)


if __name__ == "__main__":
    main()
