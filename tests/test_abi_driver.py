"""The C ABI driven from a plain C++ host program (tests/abi_driver, g++ against
include/netrep_gpu.h, as the Rcpp glue of INTEGRATION.md would), not through
Python: parity with the golden cube, explicit-shuffle validation, and the
interrupt path (MonitorProgress/checkInterrupt, src/thread-utils.cpp:49-82,
src/interrupt.cpp:9-11) returning the partial NA-padded cube
(src/permutations.cpp:375-408)."""
import os
import subprocess

import numpy as np
import pytest

import netrep_amd as N
from netrep_amd.api import RMatrix
from oracle import netrep_oracle as O

from conftest import ROOT, assert_stats_close

DRIVER = os.path.join(ROOT, "tests", "abi_driver", "abi_driver")
NA_BITS = np.uint64(0x7FF00000000007A2)


def test_driver_builds_and_links():
    """Built by __graft_entry__.build() with g++ only; runs (usage) without a GPU."""
    assert os.path.exists(DRIVER), "run make -C tests/abi_driver"
    r = subprocess.run([DRIVER], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


def write_case(d, *, data, corr, net, t_names, ma, modules, disc, n_perm, seed, null, pi=None):
    os.makedirs(d, exist_ok=True)
    n = corr.shape[0]
    s = data.shape[0] if data is not None else 0
    with open(os.path.join(d, "meta.txt"), "w") as f:
        f.write(f"{s} {n} {n_perm} {seed} {null} {int(data is not None)} {int(pi is not None)}\n")
    for name, a in (("data", data), ("corr", corr), ("net", net)):
        np.asfortranarray(a if a is not None else np.zeros((1, 1)), dtype=np.float64).T.tofile(
            os.path.join(d, f"{name}.f64"))
    for name, v in (("t_names", t_names), ("ma_names", list(ma)), ("ma_labels", list(ma.values())),
                    ("modules", modules)):
        with open(os.path.join(d, f"{name}.txt"), "w") as f:
            f.write("\n".join(map(str, v)) + "\n")
    lens = []
    parts = {"degree": [], "corr": [], "contribution": []}
    for m in modules:
        row = []
        for key in ("degree", "corr", "contribution"):
            v = np.asarray(disc.get(key, {}).get(m, np.zeros(0)), dtype=np.float64)
            parts[key].append(v)
            row.append(v.size)
        lens.append(row)
    for key, vs in parts.items():
        np.concatenate(vs + [np.zeros(0)]).tofile(os.path.join(d, f"disc_{key}.f64"))
    np.asarray(lens, dtype=np.int64).tofile(os.path.join(d, "disc_lens.i64"))
    (np.ascontiguousarray(pi, dtype=np.uint32) if pi is not None else np.zeros(1, np.uint32)).tofile(
        os.path.join(d, "pi.u32"))


def run_driver(mode, d, n_mod, n_stat, n_perm, timeout=120):
    r = subprocess.run([DRIVER, mode, d], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    rc_line = open(os.path.join(d, "rc.txt")).read().split("\n")
    nulls = np.fromfile(os.path.join(d, "nulls.f64")).reshape((n_mod, n_stat, n_perm), order="F")
    obs = np.fromfile(os.path.join(d, "observed.f64")).reshape((n_mod, n_stat), order="F")
    return int(rc_line[0]), rc_line[1], nulls, obs


def _asym_case(a, with_data, null):
    tag = "" if null == "overlap" else "_all"
    sfx = ("data" if with_data else "nodata") + tag
    modules = a["modules"].tolist()
    d_names, t_names = a["d_names"].tolist(), a["t_names"].tolist()
    ma = dict(zip(d_names, a["ma_labels"].tolist()))
    disc = {"degree": {}, "corr": {}}
    if with_data:
        disc["contribution"] = {}
    for key in list(disc):
        for m in modules:
            k = f"disc_{key}_{m}_{sfx}"
            if k in a:
                disc[key][m] = a[k]
    data = O.scale(a["t_data"]) if with_data else None
    return dict(data=data, corr=a["t_corr"], net=a["t_corr"], t_names=t_names, ma=ma, modules=modules,
                disc=disc), a["pis" + tag], a["nulls_" + sfx], a["observed_" + sfx]


@pytest.mark.gpu
@pytest.mark.parametrize("null", ["overlap", "all"])
@pytest.mark.parametrize("with_data", [True, False])
def test_driver_permutation_procedure_matches_golden(asym, tmp_path, with_data, null):
    case, pis, exp_nulls, exp_obs = _asym_case(asym, with_data, null)
    d = str(tmp_path / "case")
    write_case(d, **case, n_perm=pis.shape[0], seed=7, null=null, pi=pis)
    n_stat = 7 if with_data else 4
    rc, msg, nulls, obs = run_driver("perm", d, len(case["modules"]), n_stat, pis.shape[0])
    assert rc == 0, msg
    assert_stats_close(obs, exp_obs, what="observed via C++ driver")
    assert_stats_close(nulls, exp_nulls, what="nulls via C++ driver")


@pytest.mark.gpu
def test_bad_pi_is_rejected_before_any_device_read(asym, tmp_path):
    """An explicit shuffle with an entry >= n_null -> NR_ERR_INVALID (ADVICE r1;
    the device gather would otherwise read out of bounds)."""
    case, pis, _, _ = _asym_case(asym, True, "overlap")
    bad = pis.copy()
    bad[1, 3] = 10_000_000
    d = str(tmp_path / "bad")
    write_case(d, **case, n_perm=pis.shape[0], seed=7, null="overlap", pi=bad)
    rc, msg, _, _ = run_driver("perm", d, len(case["modules"]), 7, pis.shape[0])
    assert rc == 2 and "n_null" in msg, (rc, msg)
    # and through Python: wrong shape, and out-of-range values
    with pytest.raises(N.NetRepError):
        N.PermutationProcedure(case["disc"], RMatrix(case["data"], None, case["t_names"]),
                               RMatrix(case["corr"], case["t_names"], case["t_names"]),
                               RMatrix(case["net"], case["t_names"], case["t_names"]), case["ma"],
                               case["modules"], pis.shape[0], pi=pis[:, :-1])
    with pytest.raises(N.NetRepError) as ei:
        N.PermutationProcedure(case["disc"], RMatrix(case["data"], None, case["t_names"]),
                               RMatrix(case["corr"], case["t_names"], case["t_names"]),
                               RMatrix(case["net"], case["t_names"], case["t_names"]), case["ma"],
                               case["modules"], pis.shape[0], pi=bad)
    assert ei.value.code == 2


def _long_case():
    from netrep_amd import synthetic as S
    lay = S.make_layout(3000, np.round(np.linspace(30, 300, 10)).astype(int), 5)
    dx, dc, dn = S.numpy_dataset(lay, 100, 6)
    tx, tc, tn = S.numpy_dataset(lay, 100, 7, preserve_all=False)
    names = lay.names
    ma = dict(zip(names, lay.labels))
    mods = lay.modules
    disc = N.IntermediateProperties(N.Scale(RMatrix(dx, None, names)), RMatrix(dc, names, names),
                                    RMatrix(dn, names, names), names, ma, mods)
    return dict(data=O.scale(tx), corr=tc, net=tn, t_names=names, ma=ma, modules=mods, disc=disc)


@pytest.mark.gpu
def test_interrupt_returns_partial_cube(tmp_path):
    """The hook fires on its 3rd poll (~200 ms): the driver gets NR_ERR_CANCELLED,
    observed complete, a prefix of permutations computed (bitwise equal to an
    uninterrupted run of that prefix) and every later slice NA_real_."""
    case = _long_case()
    n_perm, seed = 400_000, 99
    d = str(tmp_path / "int")
    write_case(d, **case, n_perm=n_perm, seed=seed, null="overlap")
    M = len(case["modules"])
    rc, msg, nulls, obs = run_driver("interrupt", d, M, 7, n_perm)
    assert rc == 5 and "cancel" in msg, (rc, msg)
    assert np.isfinite(obs).all()
    bits = nulls.view(np.uint64)
    done = np.array([not (bits[:, :, p] == NA_BITS).all() for p in range(n_perm)])
    n_done = int(done.sum())
    assert 0 < n_done < n_perm, n_done
    assert done[:n_done].all() and not done[n_done:].any(), "computed slices are not a prefix"
    # the prefix equals the same permutations computed without interruption
    ref = N.PermutationProcedure(case["disc"], RMatrix(case["data"], None, case["t_names"]),
                                 RMatrix(case["corr"], case["t_names"], case["t_names"]),
                                 RMatrix(case["net"], case["t_names"], case["t_names"]), case["ma"],
                                 case["modules"], n_done, seed=seed)
    np.testing.assert_array_equal(nulls[:, :, :n_done].view(np.uint64), ref["nulls"].view(np.uint64))


@pytest.mark.gpu
def test_python_interrupt_hook(tmp_path):
    """netrep_amd.api.set_interrupt_hook: the same path from Python."""
    from netrep_amd.api import set_interrupt_hook
    case = _long_case()
    calls = {"n": 0}

    def hook():
        calls["n"] += 1
        return calls["n"] >= 2

    set_interrupt_hook(hook)
    try:
        r = N.PermutationProcedure(case["disc"], RMatrix(case["data"], None, case["t_names"]),
                                   RMatrix(case["corr"], case["t_names"], case["t_names"]),
                                   RMatrix(case["net"], case["t_names"], case["t_names"]), case["ma"],
                                   case["modules"], 400_000, seed=3)
    finally:
        set_interrupt_hook(None)
    assert r.get("interrupted") is True
    assert (r["nulls"][:, :, -1].view(np.uint64) == NA_BITS).all()


@pytest.mark.gpu
def test_shared_device_two_contexts_bitwise_equal(monkeypatch):
    """NETREP_NUM_GPUS=2 with NETREP_SHARE_DEVICE=1: two contexts on one GPU, the
    dataset uploaded once and copied device to device (nr_copy_dataset), each
    context running its contiguous chunk -- bitwise equal to one context."""
    case = _long_case()
    args = (case["disc"], RMatrix(case["data"], None, case["t_names"]),
            RMatrix(case["corr"], case["t_names"], case["t_names"]),
            RMatrix(case["net"], case["t_names"], case["t_names"]), case["ma"], case["modules"], 301)
    one = N.PermutationProcedure(*args, seed=11)
    monkeypatch.setenv("NETREP_NUM_GPUS", "2")
    monkeypatch.setenv("NETREP_SHARE_DEVICE", "1")
    two = N.PermutationProcedure(*args, seed=11)
    np.testing.assert_array_equal(one["nulls"].view(np.uint64), two["nulls"].view(np.uint64))
    np.testing.assert_array_equal(one["observed"].view(np.uint64), two["observed"].view(np.uint64))
    monkeypatch.setenv("NETREP_NUM_GPUS", "3")
    three = N.PermutationProcedure(*args, seed=11)
    np.testing.assert_array_equal(one["nulls"].view(np.uint64), three["nulls"].view(np.uint64))


@pytest.mark.gpu
def test_progress_hook_replaces_console_output(tmp_path):
    """verbose = 1 with netrep_set_progress_hook (VERDICT r2 item 3,
    MonitorProgress src/thread-utils.cpp:54-81): the hook sees BEGIN, UPDATEs
    with non-decreasing counts formatted as the reference's "%5d% completed."
    line and a final done == total update, then END -- and the library writes
    nothing to stdout / stderr itself."""
    case = _long_case()
    n_perm = 150_000
    d = str(tmp_path / "prog")
    write_case(d, **case, n_perm=n_perm, seed=5, null="overlap")
    r = subprocess.run([DRIVER, "progress", d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout == "" and r.stderr == "", (r.stdout[:200], r.stderr[:200])
    rc = int(open(os.path.join(d, "rc.txt")).read().split("\n")[0])
    assert rc == 0
    lines = [ln.split(" ", 3) for ln in open(os.path.join(d, "progress.txt")).read().splitlines()]
    events = [int(x[0]) for x in lines]
    assert events[0] == 0 and events[-1] == 2 and set(events[1:-1]) == {1}, events
    upd = [(int(x[1]), int(x[2]), x[3]) for x in lines if x[0] == "1"]
    assert len(upd) >= 2
    done = [u[0] for u in upd]
    assert done == sorted(done) and done[-1] == n_perm and all(u[1] == n_perm for u in upd)
    for dn, tot, text in upd:
        assert text == "%5d%% completed." % round(np.float32(dn) / np.float32(tot) * 100)
