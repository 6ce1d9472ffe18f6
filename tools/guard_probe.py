"""Guard-build probe outside pytest (stderr not captured): the first call of test_alignt_triangle."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tests.test_gpu_alignt import _tie_heavy
from taxi2_amd._native import Engine, tri_pairs
seqs = _tie_heavy(18, 900, 0x61)
seqs += ["ACGT" * 256, "A", "", "N" * 40, seqs[0]]
eng = Engine(0)
st = eng.upload(seqs, align=True)
a, b = tri_pairs(len(seqs))
print("launching", len(a), flush=True)
got, gsc = eng.all_pairs(st, 0, len(a), ("p", "p-gaps", "jc", "k2p"), (1, -1, -8, -1, -1, -1), with_scores=True)
print("ok", gsc[:5], flush=True)
