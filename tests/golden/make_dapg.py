"""Extract the reference's pretrained DAPG policy weights into inert .npz fixtures.

Run ONCE in the build container (it reads /root/reference; the GPU box never does):

    python tests/golden/make_dapg.py

Source: ``mj_envs_vision/algos/dapg_pretrained/{hammer,door,pen,relocate}-v0.pickle``, loaded by
the reference at ``mj_envs_vision/algos/baselines.py:67-73`` (``pickle.load``) and queried at
``:82-86`` (``get_action(obs)[1]['evaluation']`` = the network mean).

Safety: the pickles are NEVER unpickled.  No ``pickle.load`` / ``Unpickler`` runs on them and no
global named in the file is imported or called.  ``pickletools.genops`` (a pure opcode parser)
walks the stream and a small data-only interpreter builds an inert tree: every GLOBAL becomes a
``Ref`` holding the name, every REDUCE / NEWOBJ a ``Call`` record holding the name and its
arguments, BUILD attaches the state to the record.  Numbers, strings, bytes, tuples, lists and
dicts are the only live values.  Afterwards exactly three record kinds are interpreted by this
script, by name:

* ``torch.storage._load_from_bytes(b)``: ``b`` is a legacy torch-serialised storage, decoded with
  ``torch.load(io.BytesIO(b), weights_only=True)`` (the allow-listed loader);
* ``torch._utils._rebuild_tensor_v2(storage, offset, size, stride, ...)``: a strided view,
  rebuilt with numpy from those integers;
* ``numpy.core.multiarray._reconstruct`` + BUILD state ``(ver, shape, dtype, fortran, raw)``:
  ``np.frombuffer(raw)`` with the dtype string from the state.

Output ``tests/golden/dapg_<task>.npz``: ``W0 b0 W1 b1 W2 b2`` (fp64, ``nn.Linear`` layout
``[out, in]``), ``in_shift in_scale out_shift out_scale`` (the ``FCNetwork`` transformations
``mjrl.utils.fc_network``: ``out = (x - in_shift) / (in_scale + 1e-8)`` ... ``* out_scale +
out_shift``), ``log_std``, ``layer_sizes``.
"""
from __future__ import annotations

import io
import os
import pickletools
import sys

import numpy as np

REF = "/root/reference/mj_envs_vision/algos/dapg_pretrained"
OUT = os.path.dirname(os.path.abspath(__file__))
TASKS = ("hammer-v0", "door-v0", "pen-v0", "relocate-v0")


class Ref:
    """A global named by the stream (never resolved)."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"Ref({self.name})"


class Call:
    """REDUCE / NEWOBJ of a Ref (never executed); BUILD state attached in .state."""

    def __init__(self, fn, args):
        self.fn, self.args, self.state = fn, args, None
        self.items = {}     # SETITEM(S) on a dict-like record (OrderedDict())
        self.list = []      # APPENDS on a list-like record

    @property
    def name(self):
        return self.fn.name if isinstance(self.fn, Ref) else repr(self.fn)

    def __repr__(self):
        return f"Call({self.name})"


def parse(data: bytes):
    """Data-only interpretation of a pickle opcode stream (nothing is imported or called)."""
    stack, marks, memo = [], [], {}

    def pop_mark():
        m = marks.pop()
        items = stack[m:]
        del stack[m:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            marks.append(len(stack))
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "BINFLOAT", "BINUNICODE", "SHORT_BINUNICODE",
                   "BINBYTES", "SHORT_BINBYTES", "BINSTRING", "SHORT_BINSTRING"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n == "GLOBAL":
            stack.append(Ref(arg.replace(" ", ".")))
        elif n in ("REDUCE", "NEWOBJ"):
            args = stack.pop()
            fn = stack.pop()
            stack.append(Call(fn, args))
        elif n == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Call):
                raise ValueError(f"BUILD on {type(obj)}")
            obj.state = state
        elif n in ("SETITEM", "SETITEMS"):
            items = [stack.pop(), stack.pop()][::-1] if n == "SETITEM" else pop_mark()
            d = stack[-1]
            tgt = d if isinstance(d, dict) else d.items
            for i in range(0, len(items), 2):
                tgt[items[i]] = items[i + 1]
        elif n in ("APPEND", "APPENDS"):
            items = [stack.pop()] if n == "APPEND" else pop_mark()
            lst = stack[-1]
            (lst if isinstance(lst, list) else lst.list).extend(items)
        else:
            raise ValueError(f"opcode {n} not handled by the data-only interpreter")
    assert len(stack) == 1, stack
    return stack[0]


def _storage(call: Call) -> np.ndarray:
    import torch
    assert call.name == "torch.storage._load_from_bytes", call
    st = torch.load(io.BytesIO(call.args[0]), weights_only=True)
    return np.array(st.tolist(), dtype=np.float64)


def tensor(obj) -> np.ndarray:
    """Array of a tensor / parameter / ndarray record."""
    if isinstance(obj, Call) and obj.name == "torch._utils._rebuild_parameter":
        return tensor(obj.args[0])
    if isinstance(obj, Call) and obj.name == "torch._utils._rebuild_tensor_v2":
        st, off, size, stride = obj.args[:4]
        flat = _storage(st)
        if not size:
            return flat[off:off + 1].reshape(())
        return np.lib.stride_tricks.as_strided(flat[off:], shape=size,
                                               strides=[s * flat.itemsize for s in stride]).copy()
    if isinstance(obj, Call) and obj.name == "numpy.core.multiarray._reconstruct":
        _ver, shape, dt, fortran, raw = obj.state
        assert isinstance(dt, Call) and dt.name == "numpy.dtype", dt
        code = dt.args[0]
        endian = dt.state[1] if dt.state else "<"
        a = np.frombuffer(raw, dtype=np.dtype(endian + code)).reshape(shape, order="F" if fortran else "C")
        return a.astype(np.float64)
    raise TypeError(f"not a tensor record: {obj!r}")


def attrs(call: Call) -> dict:
    st = call.state
    if isinstance(st, tuple):     # (dict, slotstate)
        st = st[0]
    return st


def extract(path: str) -> dict:
    with open(path, "rb") as f:
        root = parse(f.read())
    assert isinstance(root, Call) and root.name == "mjrl.policies.gaussian_mlp.MLP", root
    a = attrs(root)
    net = a["model"]
    assert net.name == "mjrl.utils.fc_network.FCNetwork", net
    na = attrs(net)
    layers = attrs(na["_modules"].items["fc_layers"])["_modules"].items
    out = {}
    for i in range(len(layers)):
        lin = layers[str(i)]
        p = attrs(lin)["_parameters"].items
        out[f"W{i}"] = tensor(p["weight"])
        out[f"b{i}"] = tensor(p["bias"])
    sizes = [int(x) for x in na["layer_sizes"]]
    for k in ("in_shift", "in_scale", "out_shift", "out_scale"):
        # FCNetwork.forward uses the fp32 tensor attributes set by set_transformations (None in
        # the transformations dict -> zeros for a shift, ones for a scale)
        if na.get(k) is not None:
            out[k] = tensor(na[k])
        else:
            dim = sizes[0] if k.startswith("in") else sizes[-1]
            out[k] = np.zeros(dim) if "shift" in k else np.ones(dim)
        tr = na["transformations"].get(k)
        if tr is not None:
            assert np.allclose(tensor(tr), out[k], rtol=1e-6, atol=1e-6), k
    out["log_std"] = tensor(a["log_std"])
    out["layer_sizes"] = np.array(na["layer_sizes"], np.int64)
    out["min_log_std"] = np.array(float(a.get("min_log_std", -3.0)))
    return out


def main():
    for task in TASKS:
        d = extract(os.path.join(REF, f"{task}.pickle"))
        sizes = tuple(int(x) for x in d["layer_sizes"])
        for i in range(len(sizes) - 1):
            assert d[f"W{i}"].shape == (sizes[i + 1], sizes[i]), (task, i, d[f"W{i}"].shape)
        path = os.path.join(OUT, f"dapg_{task.split('-')[0]}.npz")
        np.savez(path, **d)
        print(task, sizes, "log_std", np.round(d["log_std"], 3)[:4], "->", os.path.relpath(path))


if __name__ == "__main__":
    sys.exit(main())
