"""Decoder-configuration I/O.

The reference stores a designed decoder as ``pickle.dump(self.__dict__)`` of its density-evolution
class (``AWGN_Channel_Transmission/AWGN_Discrete_Density_Evolution.py:197-206``) and the BER drivers
read the keys ``Trellis_checknodevector_a``, ``Trellis_varnodevector_a``,
``matching_vector_checknode``, ``matching_vector_varnode``, ``cardinality_T_decoder_ops``, ``imax``
(``Irregular_LDPC_Decoding/DVB-S2/BER_simulation_OpenCL.py:50-74``).

Here a configuration is written as ``.npz`` (or ``.json``) with the same keys and read back with
loaders that execute nothing (``numpy.load(allow_pickle=False)``, ``json``). A ``.pkl`` written by
the reference's own design code can be read with :func:`load_decoder_config` too: it goes through
an allow-list unpickler that reconstructs only numpy arrays / dtypes / scalars and plain Python
containers and refuses every other global (no code from the file runs). Convert once with
:func:`save_decoder_config` and keep the ``.npz``.
"""
from __future__ import annotations

import io
import json
import os
import pickle
from typing import Any, Dict

import numpy as np

from .tables import IBTables

__all__ = ["load_decoder_config", "save_decoder_config", "tables_from_config", "config_from_tables",
           "REFERENCE_KEYS"]

REFERENCE_KEYS = ("Trellis_checknodevector_a", "Trellis_varnodevector_a", "matching_vector_checknode",
                  "matching_vector_varnode", "cardinality_T_decoder_ops", "imax")

_ALLOWED_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("builtins", "complex"), ("builtins", "set"), ("builtins", "frozenset"), ("builtins", "slice"),
    ("collections", "OrderedDict"),
}


class _NumpyOnlyUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED_GLOBALS:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refused global {module}.{name}: only numpy arrays and plain containers load")


def load_decoder_config(path: str) -> Dict[str, Any]:
    """Read a decoder configuration (``.npz`` / ``.json`` / allow-listed ``.pkl``) -> dict."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npz":
        with np.load(path, allow_pickle=False) as z:
            return {k: (z[k].item() if z[k].ndim == 0 else z[k]) for k in z.files}
    if ext == ".json":
        with open(path) as fh:
            d = json.load(fh)
        return {k: (np.asarray(v) if isinstance(v, list) else v) for k, v in d.items()}
    if ext == ".pkl":
        with open(path, "rb") as fh:
            d = _NumpyOnlyUnpickler(io.BytesIO(fh.read())).load()
        if not isinstance(d, dict):
            raise ValueError("a decoder configuration pickle must hold a dict")
        return d
    raise ValueError(f"unknown decoder configuration format: {path}")


def save_decoder_config(path: str, cfg: Dict[str, Any]) -> None:
    """Write the reference keys (and any other array / scalar entries) as ``.npz`` or ``.json``."""
    ext = os.path.splitext(path)[1].lower()
    plain = {}
    for k, v in cfg.items():
        if isinstance(v, (np.ndarray, list, tuple)) or np.isscalar(v):
            plain[k] = np.asarray(v)
    if ext == ".npz":
        np.savez_compressed(path, **plain)
    elif ext == ".json":
        with open(path, "w") as fh:
            json.dump({k: v.tolist() for k, v in plain.items()}, fh)
    else:
        raise ValueError("save as .npz or .json")


def tables_from_config(cfg: Dict[str, Any], d_c_max: int, d_v_max: int, T_ch: int | None = None) -> IBTables:
    """IB tables of a configuration dict (reference key names)."""
    T = int(cfg["cardinality_T_decoder_ops"])
    Tc = int(T_ch if T_ch is not None else cfg.get("cardinality_T_channel", T))
    tb = IBTables(Tc, T, int(d_c_max), int(d_v_max), int(cfg["imax"]),
                  np.asarray(cfg["Trellis_checknodevector_a"], np.int32).ravel(),
                  np.asarray(cfg["Trellis_varnodevector_a"], np.int32).ravel(),
                  np.asarray(cfg.get("matching_vector_checknode", np.zeros(0)), np.int32).ravel(),
                  np.asarray(cfg.get("matching_vector_varnode", np.zeros(0)), np.int32).ravel())
    tb.check()
    return tb


def config_from_tables(tb: IBTables, **extra) -> Dict[str, Any]:
    cfg = {"Trellis_checknodevector_a": tb.cn, "Trellis_varnodevector_a": tb.vn,
           "matching_vector_checknode": tb.match_cn, "matching_vector_varnode": tb.match_vn,
           "cardinality_T_decoder_ops": tb.T, "cardinality_T_channel": tb.Tc, "imax": tb.imax}
    cfg.update(extra)
    return cfg
