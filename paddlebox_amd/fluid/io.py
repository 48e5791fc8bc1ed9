"""Dense checkpoint I/O (``fluid.io.save_persistables`` & co).

Reference: ``py/fluid/io.py`` (save_persistables :675, load_persistables
:1049, save_inference_model :1248).  Files hold no pickles: one ``.npy`` per
variable (``numpy.save`` / ``numpy.load(allow_pickle=False)``), or a single
safetensors file when ``filename`` is given.  Sparse (BoxPS) parameters are
saved by ``BoxWrapper.save_base/save_delta``, not here.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional

import numpy as np
import torch

from .framework import Parameter, Program, Variable, default_main_program, global_scope


def _persistables(program: Program) -> List[Variable]:
    return [v for v in program.global_block().vars.values() if v.persistable]


def _params(program: Program) -> List[Variable]:
    return [v for v in program.global_block().vars.values() if isinstance(v, Parameter)]


def _to_np(t: torch.Tensor) -> np.ndarray:
    return t.detach().float().cpu().numpy() if t.dtype == torch.bfloat16 else t.detach().cpu().numpy()


def save_vars(executor, dirname: str, main_program: Optional[Program] = None, vars: Optional[Iterable] = None,  # noqa: A002
              predicate=None, filename: Optional[str] = None, scope=None):
    program = main_program or default_main_program()
    scope = scope or global_scope()
    vs = list(vars) if vars is not None else [v for v in program.global_block().vars.values()
                                              if predicate is None or predicate(v)]
    os.makedirs(dirname, exist_ok=True)
    arrays = {}
    for v in vs:
        name = v if isinstance(v, str) else v.name
        if name not in scope:
            continue
        arrays[name] = _to_np(scope.get(name))
    if filename:
        from safetensors.numpy import save_file

        save_file({k: np.ascontiguousarray(a) for k, a in arrays.items()}, os.path.join(dirname, filename))
    else:
        for name, a in arrays.items():
            np.save(os.path.join(dirname, name + ".npy"), a, allow_pickle=False)
    return list(arrays)


def load_vars(executor, dirname: str, main_program: Optional[Program] = None, vars: Optional[Iterable] = None,  # noqa: A002
              predicate=None, filename: Optional[str] = None, scope=None):
    program = main_program or default_main_program()
    scope = scope or global_scope()
    vs = list(vars) if vars is not None else [v for v in program.global_block().vars.values()
                                              if predicate is None or predicate(v)]
    names = [v if isinstance(v, str) else v.name for v in vs]
    if filename:
        from safetensors.numpy import load_file

        arrays = load_file(os.path.join(dirname, filename))
    else:
        arrays = {}
        for n in names:
            p = os.path.join(dirname, n + ".npy")
            if os.path.exists(p):
                arrays[n] = np.load(p, allow_pickle=False)
    loaded = []
    for n in names:
        if n in arrays:
            t = torch.as_tensor(arrays[n])
            if n in scope:
                cur = scope.get(n)
                with torch.no_grad():
                    cur.copy_(t.reshape(cur.shape).to(cur.device, cur.dtype))
            else:
                scope.set(n, t)
            loaded.append(n)
    return loaded


_OPT_FILE = "__optimizer_state__.safetensors"


def save_persistables(executor, dirname: str, main_program: Optional[Program] = None, filename=None, scope=None):
    """Persistable variables plus the optimizer state of the executor's
    training session for the program (Adam moments / beta powers under the
    reference's ``<param>_moment1_0``-style names; one safetensors file)."""
    program = main_program or default_main_program()
    saved = save_vars(executor, dirname, program, _persistables(program), filename=filename, scope=scope)
    sessions = executor.sessions_for(program) if hasattr(executor, "sessions_for") else []
    if sessions:
        from safetensors.numpy import save_file

        st = {k: np.ascontiguousarray(_to_np(v)) for k, v in sessions[0].optimizer_state().items()}
        if st:
            # format marker: beta-pow accumulators hold beta^(t+1) (the
            # reference convention); files without it hold beta^t
            save_file(st, os.path.join(dirname, _OPT_FILE), metadata={"beta_pow_convention": "reference"})
            saved += list(st)
    return saved


def load_persistables(executor, dirname: str, main_program: Optional[Program] = None, filename=None,
                      scope=None):
    """Load persistables; optimizer state goes into the live training session
    when the program already ran, else into the scope, where the session
    picks it up when it builds its optimizers (exact resume)."""
    program = main_program or default_main_program()
    loaded = load_vars(executor, dirname, program, _persistables(program), filename=filename, scope=scope)
    p = os.path.join(dirname, _OPT_FILE)
    if os.path.exists(p):
        from safetensors import safe_open
        from safetensors.numpy import load_file

        st = load_file(p)
        with safe_open(p, "np") as f:
            meta = f.metadata() or {}
        # written before the format marker existed: raw beta^t powers
        ref_pows = meta.get("beta_pow_convention") == "reference"
        sessions = executor.sessions_for(program) if hasattr(executor, "sessions_for") else []
        if sessions:
            sessions[0].load_optimizer_state(st, reference_pows=ref_pows)
        else:
            sc = scope or global_scope()
            for k, a in st.items():
                sc.set(k, torch.as_tensor(a))
            sc.set("@beta_pow_convention@", torch.tensor(1 if ref_pows else 0))
        loaded += list(st)
    return loaded


def save_params(executor, dirname: str, main_program: Optional[Program] = None, filename=None):
    program = main_program or default_main_program()
    return save_vars(executor, dirname, program, _params(program), filename=filename)


def load_params(executor, dirname: str, main_program: Optional[Program] = None, filename=None):
    program = main_program or default_main_program()
    return load_vars(executor, dirname, program, _params(program), filename=filename)


def save_inference_model(dirname: str, feeded_var_names: List[str], target_vars: List[Variable], executor,
                         main_program: Optional[Program] = None, model_filename=None, params_filename=None,
                         export_for_deployment=True, program_only=False):
    """Writes ``__model__.json`` (op list of the pruned forward program) and
    the parameters."""
    program = (main_program or default_main_program()).clone(for_test=True)
    os.makedirs(dirname, exist_ok=True)
    desc = {
        "feed": list(feeded_var_names),
        "fetch": [v.name for v in target_vars],
        "vars": {n: {"shape": list(v.shape), "dtype": v.dtype, "lod_level": v.lod_level,
                     "persistable": v.persistable, "is_data": v.is_data,
                     "param": isinstance(v, Parameter)} for n, v in program.global_block().vars.items()},
        "ops": [{"type": op.type, "inputs": {k: [v.name for v in vs] for k, vs in op.inputs.items()},
                 "outputs": {k: [v.name for v in vs] for k, vs in op.outputs.items()},
                 "attrs": {k: a for k, a in op.attrs.items() if isinstance(a, (int, float, str, bool, list))}}
                for op in program.global_block().ops],
    }
    with open(os.path.join(dirname, model_filename or "__model__.json"), "w") as f:
        json.dump(desc, f)
    if not program_only:
        save_params(executor, dirname, program, params_filename)
    return desc["fetch"]


def load_inference_model(dirname: str, executor, model_filename=None, params_filename=None):
    """Rebuilds the forward program from ``__model__.json`` and loads its
    parameters; returns ``(program, feed_names, fetch_vars)``."""
    from .framework import Program, Parameter as P

    with open(os.path.join(dirname, model_filename or "__model__.json")) as f:
        desc = json.load(f)
    prog = Program()
    blk = prog.global_block()
    for n, v in desc["vars"].items():
        if v["param"]:
            blk.vars[n] = P(blk, n, v["shape"], v["dtype"])
        else:
            blk.create_var(n, v["shape"], v["dtype"], v["lod_level"], v["persistable"], is_data=v["is_data"])
    for op in desc["ops"]:
        blk.append_op(op["type"], {k: [blk.var(x) for x in vs] for k, vs in op["inputs"].items()},
                      {k: [blk.var(x) for x in vs] for k, vs in op["outputs"].items()}, op["attrs"])
    prog._is_test = True
    load_params(executor, dirname, prog, params_filename)
    return prog, desc["feed"], [blk.var(n) for n in desc["fetch"]]
