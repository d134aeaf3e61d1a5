"""The guided-tour notebook (notebooks/hyperspace_amd_tour.ipynb) runs top to bottom on the host
executor (the reference ships "Hitchhiker's Guide" notebooks; this one is executed in CI)."""
import contextlib
import io
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tour_notebook_executes(monkeypatch):
    monkeypatch.setenv("HS_TOUR_DEVICE", "cpu")
    nb = json.load(open(os.path.join(ROOT, "notebooks", "hyperspace_amd_tour.ipynb")))
    env: dict = {}
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        for cell in nb["cells"]:
            if cell["cell_type"] == "code":
                exec(compile("".join(cell["source"]), "<notebook>", "exec"), env)
    text = out.getvalue()
    assert "Hyperspace(Type: CI, Name: empSalary" in text or "empSalary" in text
    assert "new0" in text and "new1" in text
