"""Generate tests/golden/*.tbl from the reference's known-answer tables.

The reference's state-machine tests (src/state_machine.zig:2032-2575) are tables
of rows (`account ...`, `transfer ...`, `setup`, `tick`, `commit`, `lookup_*`)
fed to `check()` (:1867-2030) and parsed by src/testing/table.zig:8-100.
This script copies only the table ROWS (the data: inputs + expected results)
into one .tbl file per `check(...)` call; the harness that interprets them is
our own (tests/table.py).  Run it in the build container, where /root/reference
exists; the generated files are committed so the GPU box never needs it.

    python tests/golden/extract_tables.py /root/reference/src/state_machine.zig
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main(path):
    lines = open(path, encoding="utf-8").read().split("\n")
    test_name, check_no, out = None, 0, []
    i = 0
    while i < len(lines):
        m = re.match(r'^test "(.*)" \{', lines[i])
        if m:
            test_name, check_no = m.group(1), 0
        if lines[i].strip() == "try check(" and test_name is not None:
            start = i + 1
            check_no += 1
            rows = []
            j = i + 1
            while not lines[j].strip().startswith(");"):
                s = lines[j].strip()
                if s.startswith("\\\\"):
                    row = s[2:]
                    row = row.split("//")[0].rstrip()
                    rows.append(row.strip())
                j += 1
            out.append((test_name, check_no, start, rows))
            i = j
        i += 1
    for name, k, line, rows in out:
        slug = re.sub(r"[^a-z0-9]+", "_", name.replace("¬", "not ").lower()).strip("_")
        fname = f"{slug}_{k}.tbl"
        with open(os.path.join(HERE, fname), "w") as f:
            f.write(f"# source: src/state_machine.zig:{line}  test \"{name}\"  check #{k}\n")
            for r in rows:
                f.write(r + "\n")
        print(fname, len(rows))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/state_machine.zig")
