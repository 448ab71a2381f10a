"""Crude undefined-name check for the package (no pyflakes in the image):
every Name read must be bound somewhere in its module (assignment, def,
class, import, parameter, comprehension / except / with target) or be a
builtin. Catches leftovers of removed helpers in GPU-only code paths that the
CPU test suite never executes.

    python tools/check_names.py [paths...]
"""
import ast
import builtins
import pathlib
import sys


def bound_names(tree):
    out = set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__path__", "__package__"}
    for n in ast.walk(tree):
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                out.add((a.asname or a.name).split(".")[0])
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
    return out


def main(paths):
    bad = 0
    for root in paths:
        for f in sorted(pathlib.Path(root).rglob("*.py")) if pathlib.Path(root).is_dir() else [pathlib.Path(root)]:
            tree = ast.parse(f.read_text(), str(f))
            ok = bound_names(tree)
            for n in ast.walk(tree):
                if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id not in ok:
                    print(f"{f}:{n.lineno}: undefined name {n.id!r}")
                    bad += 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["distributed_compute_pytorch_amd", "bench.py", "__graft_entry__.py",
                                   "tools", "tests", "examples"]))
