"""Extract the reference's hot-path test VECTORS (data only) into JSON fixtures.

Run once in the build container (``python tests/golden/make_golden_from_reference.py``);
the reference tree does not exist on the GPU box, so the JSON it writes is committed.

Sources (read as text with ``ast``; nothing from the reference is imported or executed):
  * ``tests/test_align.py:49-163``   -> align_tests.json   (input pair, accepted solutions, 6 scores)
  * ``tests/test_align.py:166-203``  -> align_tests_failing.json (xfail rows, kept for information)
  * ``tests/test_distances.py:515-521`` -> metric_tests.json (label, x, y, expected d or null)
  * ``tests/test_pairs.py:92-112``   -> fromProduct order is restated directly in tests
"""

from __future__ import annotations

import ast
import json
from pathlib import Path

REF = Path("/root/reference/tests")
OUT = Path(__file__).parent

SCORE_KEYS = [
    "match_score",
    "mismatch_score",
    "internal_open_gap_score",
    "internal_extend_gap_score",
    "end_open_gap_score",
    "end_extend_gap_score",
]


def _align_rows(tree: ast.Module, name: str) -> list[dict]:
    for node in tree.body:
        if isinstance(node, ast.Assign) and node.targets[0].id == name:
            rows = []
            for call in node.value.elts:
                args = [ast.literal_eval(a) for a in call.args]
                inp, sols = args[0], args[1]
                scores = args[2] if len(args) > 2 else (1, -1, -8, -1, -1, -1)
                rows.append(
                    dict(
                        x=inp[0],
                        y=inp[1],
                        solutions=[list(s) for s in sols],
                        scores=dict(zip(SCORE_KEYS, scores)),
                    )
                )
            return rows
    raise KeyError(name)


def _metric_rows(tree: ast.Module) -> list[dict]:
    for node in tree.body:
        if isinstance(node, ast.Assign) and node.targets[0].id == "metric_tests":
            rows = []
            for call in node.value.elts:
                metric = call.args[0].func.attr  # DistanceMetric.<Class>()
                x = ast.literal_eval(call.args[1])
                y = ast.literal_eval(call.args[2])
                d = call.args[3]
                if isinstance(d, ast.Constant) and d.value is None:
                    val = None
                else:  # e.g. 1.0 / 8.0
                    val = eval(compile(ast.Expression(d), "<d>", "eval"), {}, {})
                rows.append(dict(metric=metric, x=x, y=y, d=val))
            return rows
    raise KeyError("metric_tests")


def main() -> None:
    align = ast.parse((REF / "test_align.py").read_text())
    (OUT / "align_tests.json").write_text(
        json.dumps(_align_rows(align, "align_tests"), indent=1) + "\n"
    )
    (OUT / "align_tests_failing.json").write_text(
        json.dumps(_align_rows(align, "align_tests_failing"), indent=1) + "\n"
    )
    dist = ast.parse((REF / "test_distances.py").read_text())
    (OUT / "metric_tests.json").write_text(
        json.dumps(_metric_rows(dist), indent=1) + "\n"
    )


if __name__ == "__main__":
    main()
