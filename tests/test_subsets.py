"""VersusAll summary.tsv and subset statistics (versus_all.py:57-350, 605-684, 754-768).

Expected text is rebuilt here in the reference's own shape -- one SubsetDistance per (pair,
metric), DistanceHandler.Linear line grouping, DistanceAggregator dicts (oracle A11), the
Subset*StatisticsHandler rules -- from the same value matrix.  No reference fixture covers these
files: parity is pinned to the restated code, not to reference outputs."""

from __future__ import annotations

from itertools import groupby

import numpy as np
import pytest

from oracle import restatement as R

CMP = {  # SubsetDistance.get_comparison_type, versus_all.py:255-271
    (None, None): "no info", (None, True): "intra-species", (None, False): "inter-species",
    (False, None): "inter-genus", (False, True): "inter-genus", (False, False): "inter-genus",
    (True, None): "intra-genus", (True, True): "intra-species", (True, False): "inter-species",
}


def txt(v, fmt="{:.4f}", missing="NA"):
    return missing if v is None else fmt.format(v)


def value_fn(A):
    def value(i, j, k):
        v = A[i, j, k]
        return float(v) if np.isfinite(v) else None

    return value


def exp_summary(seqs, A, metrics, genera, species, fmt="{:.4f}", missing="NA") -> str:
    value = value_fn(A)
    items = []  # SubsetDistance stream: (x, y, metric, d, genera pair, species pair)
    for i, x in enumerate(seqs):
        for j, y in enumerate(seqs):
            g = (genera.get(x.id, None), genera.get(y.id, None)) if genera else None
            s = (species.get(x.id, None), species.get(y.id, None)) if species else None
            for k, m in enumerate(metrics):
                items.append((x, y, m, value(i, j, k), g, s))
    out = []
    for n, (_, grp) in enumerate(groupby(items, key=lambda t: (t[0].id, t[1].id))):
        line = list(grp)
        x, y, _, _, g, s = line[0]
        if n == 0:
            out.append("\t".join(("seqid (query 1)", "seqid (query 2)", *[str(t[2]) for t in line],
                                  *[k + " (query 1)" for k in x.extras], *[k + " (query 2)" for k in y.extras],
                                  "genus (query 1)", "species (query 1)", "genus (query 2)", "species (query 2)",
                                  "comparison_type")))
        sg = (g[0] == g[1]) if g else None
        ss = (s[0] == s[1]) if s else None
        out.append("\t".join((x.id, y.id, *[txt(t[3], fmt, missing) for t in line],
                              *[v if v is not None else missing for v in x.extras.values()],
                              *[v if v is not None else missing for v in y.extras.values()],
                              (g[0] if g else None) or "-", (s[0] if s else None) or "-",
                              (g[1] if g else None) or "-", (s[1] if s else None) or "-", CMP[(sg, ss)])))
    return "".join(line + "\n" for line in out)


def exp_subsets(ids, A, metrics, partition, fmt="{:.4f}", template="{mean} ({min}-{max})") -> dict:
    aggs = R.subset_aggregates(ids, partition, value_fn(A), len(metrics))

    def stats(acc):  # SimpleAggregator.calculate
        s, mn, mx, c = acc
        return (None, None, None, 0) if not c else (s / c, mn, mx, c)

    labels = [f"{m} {s}" for m in metrics for s in ("mean", "min", "max")]
    pairs, ident = [], []
    for (a, b), accs in aggs.items():
        row = [txt(v, fmt) for acc in accs for v in stats(acc)[:3]]
        na, nb = "?" if a is None else a, "?" if b is None else b
        if a == b:
            ident.append("\t".join((na, *row)))
        else:
            pairs.append("\t".join((na, nb, *row)))
    files = {
        "linear/pairs.tsv": "".join(ln + "\n" for ln in (["\t".join(("target", "query", *labels))] + pairs if pairs else [])),
        "linear/identity.tsv": "".join(ln + "\n" for ln in (["\t".join(("target", *labels))] + ident if ident else [])),
    }
    for k, m in enumerate(metrics):
        rows = []
        for a, grp in groupby(aggs.items(), key=lambda kv: kv[0][0]):
            grp = list(grp)
            if not rows:
                rows.append("\t".join(("", *["?" if b is None else b for (_, b), _ in grp])))
            cells = []
            for _, accs in grp:
                mean, mn, mx, c = stats(accs[k])
                cells.append("NA" if not c else template.format(mean=txt(mean, fmt), min=txt(mn, fmt), max=txt(mx, fmt)))
            rows.append("\t".join(("?" if a is None else a, *cells)))
        files[f"matricial/{m}.tsv"] = "".join(r + "\n" for r in rows)
    return files


def random_case(seed, n, m, dup_ids=False):
    from taxi2_amd.sequences import Sequence

    rng = np.random.default_rng(seed)
    A = rng.random((n, n, m)) * 0.3
    A[rng.random((n, n, m)) < 0.15] = np.nan
    A[rng.random((n, n, m)) < 0.05] = 0.0
    ids = [f"s{k}" for k in range(n)]
    if dup_ids and n > 3:
        ids[2] = ids[1]
    seqs = [Sequence(i, "ACGT", {"voucher": f"v{k}", "organism": None if k % 5 == 0 else f"o{k}"})
            for k, i in enumerate(ids)]
    species = {i: f"sp{int(rng.integers(0, 4))}" for i in ids if rng.random() > 0.2}
    species[ids[0]] = ""  # empty subset label: "-" in the summary, "" in the subset files
    genera = {i: ("gA" if (v or "x") < "sp2" else "gB") for i, v in species.items()}
    return seqs, A, species, genera


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_subset_aggregate_native_vs_oracle(seed):
    from taxi2_amd._native import subset_aggregate
    from taxi2_amd.tasks.subsets import subset_codes

    seqs, A, species, _ = random_case(seed, 37, 3)
    ids = [s.id for s in seqs]
    code, subsets = subset_codes(ids, species)
    want = R.subset_aggregates(ids, species, value_fn(A), 3)
    assert list(want) == [(a, b) for a in subsets for b in subsets]  # key order
    for threads in (1, 3):
        got = subset_aggregate(A, code, len(subsets), threads)
        for (a, b), accs in want.items():
            ia, ib = subsets.index(a), subsets.index(b)
            for k, (s, mn, mx, c) in enumerate(accs):
                assert got.count[ia, ib, k] == c
                assert got.sum[ia, ib, k] == s  # bit-exact: same summation order
                if c:
                    assert got.min[ia, ib, k] == mn and got.max[ia, ib, k] == mx


@pytest.mark.parametrize("seed,dup", [(3, False), (4, True)])
def test_summary_handler_text(tmp_path, seed, dup):
    """Host (handler-shaped) summary writer: line merging for repeated adjacent ids, missing
    extras, absent / partial partitions."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.tasks.subsets import write_summary

    seqs, A, species, genera = random_case(seed, 9, 2, dup)
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor()]
    for g, s in ((None, None), (genera, None), (None, species), (genera, species)):
        p = tmp_path / "summary.tsv"
        write_summary(p, seqs, A, metrics, g, s, "{:.4f}", "NA", eng=None)
        assert p.read_text() == exp_summary(seqs, A, metrics, g, s)


def test_subset_statistics_files(tmp_path):
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.tasks.subsets import aggregate, write_subset_statistics

    seqs, A, species, _ = random_case(5, 23, 2)
    A[:, :, 1][np.array([s.id for s in seqs]) == "s3"] = np.nan  # a subset row with some empty stats
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.Kimura2P()]
    ids = [s.id for s in seqs]
    write_subset_statistics(tmp_path / "sp", aggregate(A, ids, species), metrics, "{:.4f}", "{mean} ({min}-{max})")
    for name, text in exp_subsets(ids, A, metrics, species).items():
        assert (tmp_path / "sp" / name).read_text() == text, name


@pytest.mark.gpu
@pytest.mark.parametrize("pct,partitions", [(False, True), (True, True), (False, False)])
def test_versus_all_summary_and_subsets(tmp_path, engine, oracle_c, pct, partitions):
    """VersusAll end to end: summary.tsv through the GPU formatter (unique ids) and the subset
    statistics, against the oracle's distances."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.partitions import Partition
    from taxi2_amd.sequences import Sequences
    from taxi2_amd.tasks import VersusAll
    from tests.test_gpu_tasks import expected_versus_all, read_tab

    seqs = read_tab("Taxi2test1_120.tab")[:40]
    species = {s.id: s.extras["organism"] for s in seqs[::2]}  # half the ids missing -> None subset
    genera = Partition({i: v.split(" ")[0] for i, v in species.items()})
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.UncorrectedWithGaps(), DistanceMetric.JukesCantor(),
               DistanceMetric.Kimura2P()]
    task = VersusAll()
    task.engine = engine
    task.progress_handler = None
    task.work_dir = tmp_path / "out"
    task.input.sequences = Sequences(seqs)
    if partitions:
        task.input.species = Partition(species)
        task.input.genera = genera
    task.params.pairs.write = False
    task.params.format.percentage_multiply = pct
    task.start()
    work, D = expected_versus_all(seqs, ("p", "p-gaps", "jc", "k2p"), True, oracle_c)
    A = D * 100.0 if pct else D
    g, s = (genera, species) if partitions else (None, None)
    assert (tmp_path / "out/summary.tsv").read_text() == exp_summary(work, A, metrics, g, s)
    ids = [w.id for w in work]
    if partitions:
        for part, name in ((genera, "genera"), (species, "species")):
            for rel, text in exp_subsets(ids, A, metrics, part).items():
                assert (tmp_path / "out/subsets" / name / rel).read_text() == text, (name, rel)
    else:
        assert not (tmp_path / "out/subsets").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [6, 7])
def test_summary_gpu_formatter(tmp_path, engine, seed, monkeypatch):
    """taxi2_format_summary (unique ids) == the handler-shaped text: missing extras, empty subset
    labels, ids missing from a partition, every partition combination, row chunking."""
    from taxi2_amd.distances import DistanceMetric
    from taxi2_amd.tasks import subsets as S

    seqs, A, species, genera = random_case(seed, 31, 3)
    A[0, 1, 0] = -0.0
    metrics = [DistanceMetric.Uncorrected(), DistanceMetric.JukesCantor(), DistanceMetric.Kimura2P()]
    monkeypatch.setattr(S, "SUMMARY_CHUNK_VALUES", 31 * 3 * 4)  # 4 rows per call
    for g, s in ((None, None), (genera, None), (None, species), (genera, species)):
        p = tmp_path / "summary.tsv"
        S.write_summary(p, seqs, A, metrics, g, s, "{:.4f}", "NA", eng=engine)
        assert p.read_text() == exp_summary(seqs, A, metrics, g, s)
