#!/usr/bin/env python
"""Minimal lint gate (no third-party linters in the image): flags names a function reads that
are defined nowhere — not local, not enclosing, not module-level, not a builtin — using the
compiler's own symbol tables.  Catches the NameError class of bug (a dropped import) before a
GPU run does.  Usage: python scripts/lint_names.py [paths...]; exit 1 on findings."""
import builtins
import os
import sys
import symtable


def _module_names(top: symtable.SymbolTable) -> set:
    return {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()
            or s.is_namespace()}


def check_file(path: str) -> list:
    src = open(path, encoding="utf-8").read()
    try:
        top = symtable.symtable(src, path, "exec")
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: syntax error {e.msg}"]
    defined = _module_names(top) | set(dir(builtins)) | {"__file__", "__name__", "__doc__",
                                                          "__spec__", "__path__", "__builtins__"}
    if "__getattr__" in defined:
        return []
    out = []

    def walk(t: symtable.SymbolTable):
        for s in t.get_symbols():
            if t.get_type() != "module" and s.is_referenced() and s.is_global() and \
                    not s.is_declared_global() and s.get_name() not in defined:
                out.append(f"{path}: {t.get_name()}() uses undefined name {s.get_name()!r}")
        for c in t.get_children():
            walk(c)
    walk(top)
    return out


def main(argv):
    roots = argv or ["hyperspace_amd", "tests", "bench.py", "__graft_entry__.py", "benchmarks",
                     "scripts"]
    bad = []
    for r in roots:
        if os.path.isfile(r):
            bad += check_file(r)
            continue
        for d, _, fs in os.walk(r):
            for f in fs:
                if f.endswith(".py"):
                    bad += check_file(os.path.join(d, f))
    for b in bad:
        print(b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
