"""Golden-vector container: an OCPQP, the call arguments and the reference outputs in one .npz.

Lists of per-stage arrays are stored flattened with an offsets array (``<name>`` + ``<name>__off``);
everything is plain float64 / int32 / unicode (loadable with ``allow_pickle=False``).
"""
from __future__ import annotations

import os

import numpy as np

from .ocp import OCPQP

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _put_list(d, name, lst, dtype=np.float64):
    arrs = [np.ascontiguousarray(a, dtype=dtype).reshape(-1) for a in lst]
    off = np.zeros(len(arrs) + 1, dtype=np.int64)
    for i, a in enumerate(arrs):
        off[i + 1] = off[i] + a.size
    d[name] = np.concatenate(arrs) if arrs else np.zeros(0, dtype=dtype)
    d[name + "__off"] = off


def _get_list(z, name):
    flat, off = z[name], z[name + "__off"]
    return [flat[off[i]:off[i + 1]].copy() for i in range(len(off) - 1)]


def save_case(name, kind, qp: OCPQP, args: dict, outputs: dict, extra: dict | None = None) -> str:
    d = {"kind": np.array(kind), "N": np.array(qp.N)}
    for f in ("nx", "nu", "nb", "ng"):
        d[f] = np.asarray(getattr(qp, f), dtype=np.int32)
    _put_list(d, "idxb", qp.idxb, np.int32)
    _put_list(d, "BAbt", qp.BAbt)
    _put_list(d, "RSQrq", qp.RSQrq)
    _put_list(d, "d", qp.d)
    _put_list(d, "DCt", qp.DCt if qp.DCt else [])
    for k, v in args.items():
        d["arg_" + k] = np.array(float(v))
    for k, v in outputs.items():
        if isinstance(v, (list, tuple)):
            _put_list(d, "out_" + k, v)
        else:
            d["out_" + k] = np.asarray(v)
    for k, v in (extra or {}).items():
        _put_list(d, "in_" + k, v)
    os.makedirs(GOLDEN_DIR, exist_ok=True)
    path = os.path.join(GOLDEN_DIR, name + ".npz")
    np.savez_compressed(path, **d)
    return path


class Case:
    def __init__(self, path):
        self.path = path
        self.name = os.path.basename(path)[:-4]
        z = np.load(path, allow_pickle=False)
        self.kind = str(z["kind"])
        N = int(z["N"])
        self.qp = OCPQP(N, z["nx"].copy(), z["nu"].copy(), z["nb"].copy(), z["ng"].copy(), _get_list(z, "idxb"),
                        _get_list(z, "BAbt"), _get_list(z, "RSQrq"), _get_list(z, "d"), _get_list(z, "DCt"), None)
        self.qp.idxb = [a.astype(np.int32) for a in self.qp.idxb]
        self.args = {k[4:]: float(z[k]) for k in z.files if k.startswith("arg_")}
        self.out, self.inp = {}, {}
        for k in z.files:
            if k.endswith("__off"):
                continue
            if k.startswith("out_"):
                self.out[k[4:]] = _get_list(z, k) if (k + "__off") in z.files else z[k].copy()
            elif k.startswith("in_"):
                self.inp[k[3:]] = _get_list(z, k)

    def fresh_qp(self) -> OCPQP:
        return self.qp.copy()


def load_all(kind: str | None = None):
    if not os.path.isdir(GOLDEN_DIR):
        return []
    cases = [Case(os.path.join(GOLDEN_DIR, f)) for f in sorted(os.listdir(GOLDEN_DIR)) if f.endswith(".npz")]
    return [c for c in cases if kind is None or c.kind == kind]
