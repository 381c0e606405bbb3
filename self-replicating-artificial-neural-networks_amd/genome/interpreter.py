"""Safe genome interpreter: SeRANN source code -> :class:`OrganismIR`.

The reference builds organisms with ``exec(source_code)`` against Keras 2.6 layers and treats any
exception as "invalid" (common/logic.py:17-35, experiment_worker.py:232-239).  Here the source is
parsed with :mod:`ast` (no ``exec``) and evaluated by a whitelist interpreter that reproduces the
Python and Keras-2.6 semantics reachable from the genome vocabulary:

* statements: assignments (chained ``a=b=...`` and tuple unpacking), bare expressions;
* expressions: names, int/float/str constants, tuples/lists, calls with positional and keyword
  arguments, unary minus, binary minus, ``==``/``!=``;
* callables: ``Dense Conv2D Conv1D MaxPool2D BatchNormalization Reshape concatenate`` with the
  Keras argument normalisation rules (``normalize_tuple``, ``int(units)``, activation lookup,
  allowed keyword arguments, positional-argument order);
* shape inference with Keras rules: valid padding, ``Conv`` min-rank, ``MaxPool2D`` rank 4,
  ``Reshape`` unknown-dimension fixing, ``Concatenate`` shape matching.

Documented decisions where Keras 2.6 behaviour cannot be pinned without TensorFlow
("parity unpinned", see docs/genome.md): zero-sized outputs, zero/negative ``units``/``filters``,
attribute access, subscripts, re-use of one layer object on two inputs (weight sharing) and
``BatchNormalization()(x, training)`` are reported invalid.
"""
from __future__ import annotations

import ast
import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

from .ir import ACTIVATIONS, Node, OrganismIR


class GenomeError(Exception):
    """Raised for any source code that would fail to build in the reference."""


# ------------------------------------------------------------------------------------------------
# runtime values
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class Tensor:
    node: int
    shape: Tuple[int, ...]

    @property
    def ndim(self) -> int:            # rank including batch
        return len(self.shape) + 1


class LayerFactory:
    def __init__(self, kind: str):
        self.kind = kind

    def __repr__(self):
        return f"<{self.kind}>"


class ConcatenateFn:
    pass


class LayerObject:
    def __init__(self, kind: str, cfg: Dict[str, Any]):
        self.kind = kind
        self.cfg = cfg
        self.calls = 0


_ALLOWED_BASE_KW = {"input_dim", "input_shape", "batch_input_shape", "batch_size", "weights",
                    "activity_regularizer", "autocast", "implementation", "trainable", "name",
                    "dtype", "dynamic"}

# positional parameter order of each layer constructor (Keras 2.6 signatures); parameters beyond the
# supported prefix can only receive values that Keras rejects (initializers/regularizers/padding),
# so extra positionals make the organism invalid.
_SIGNATURES = {
    "Dense": ["units", "activation", "use_bias"],
    "Conv2D": ["filters", "kernel_size", "strides"],
    "Conv1D": ["filters", "kernel_size", "strides"],
    "MaxPool2D": ["pool_size", "strides"],
    "BatchNormalization": ["axis", "momentum", "epsilon", "center", "scale"],
    "Reshape": ["target_shape"],
}
_KWARGS = {
    "Dense": {"units", "activation", "use_bias", "kernel_initializer", "bias_initializer",
              "kernel_regularizer", "bias_regularizer", "kernel_constraint", "bias_constraint"},
    "Conv2D": {"filters", "kernel_size", "strides", "padding", "data_format", "dilation_rate",
               "groups", "activation", "use_bias"},
    "Conv1D": {"filters", "kernel_size", "strides", "padding", "data_format", "dilation_rate",
               "groups", "activation", "use_bias"},
    "MaxPool2D": {"pool_size", "strides", "padding", "data_format"},
    "BatchNormalization": {"axis", "momentum", "epsilon", "center", "scale"},
    "Reshape": {"target_shape"},
}
_DEFAULTS = {
    "Dense": {"activation": None, "use_bias": True},
    "Conv2D": {"strides": 1, "activation": None, "use_bias": True},
    "Conv1D": {"strides": 1, "activation": None, "use_bias": True},
    "MaxPool2D": {"pool_size": 2, "strides": None},
    "BatchNormalization": {"axis": -1, "momentum": 0.99, "epsilon": 1e-3, "center": True, "scale": True},
    "Reshape": {},
}
_REQUIRED = {"Dense": ["units"], "Conv2D": ["filters", "kernel_size"], "Conv1D": ["filters", "kernel_size"],
             "Reshape": ["target_shape"]}


def _is_int(v) -> bool:
    return isinstance(v, int) and not isinstance(v, bool)


def _to_int(v, what: str) -> int:
    """``int(x) if not isinstance(x, int) else x`` as Keras does for units/filters."""
    if isinstance(v, (Tensor, LayerObject, LayerFactory, ConcatenateFn, tuple, list)) or v is None:
        raise GenomeError(f"{what}: cannot convert {v!r} to int")
    try:
        return int(v)
    except (TypeError, ValueError) as e:
        raise GenomeError(f"{what}: {e}")


def _normalize_tuple(value, n: int, what: str) -> Tuple[int, ...]:
    """keras.utils.conv_utils.normalize_tuple."""
    if _is_int(value) or isinstance(value, bool):
        return (int(value),) * n
    if isinstance(value, (tuple, list)):
        if len(value) != n:
            raise GenomeError(f"{what} must be a tuple of {n} integers")
        if not all(_is_int(v) for v in value):
            raise GenomeError(f"{what} must contain integers")
        return tuple(int(v) for v in value)
    raise GenomeError(f"{what} must be an int or tuple")


def _activation(v) -> str:
    if v is None:
        return "linear"
    if isinstance(v, str):
        if v in ACTIVATIONS:
            return v
        raise GenomeError(f"unknown activation {v!r}")
    raise GenomeError(f"could not interpret activation {v!r}")


def _to_float(v, what: str) -> float:
    if isinstance(v, (int, float)):           # bools included
        return float(v)
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError as e:
            raise GenomeError(f"{what}: {e}")
    raise GenomeError(f"{what}: cannot convert {v!r} to float")


# ------------------------------------------------------------------------------------------------
# interpreter
# ------------------------------------------------------------------------------------------------
class _Builder:
    def __init__(self, image_shape: Tuple[int, int], genotype_size: int):
        self.nodes: List[Node] = []
        self.x = self._add("input", [], (image_shape[0], image_shape[1], 1), {"name": "X"})
        self.g = self._add("input", [], (genotype_size, 1), {"name": "g"})

    def _add(self, op, inputs, shape, attrs) -> Tensor:
        if any(d <= 0 for d in shape):
            raise GenomeError(f"{op}: zero-sized or negative output shape {shape}")
        nid = len(self.nodes)
        self.nodes.append(Node(nid, op, list(inputs), tuple(int(s) for s in shape), dict(attrs)))
        return Tensor(nid, tuple(int(s) for s in shape))

    # -- layer application ---------------------------------------------------------------------
    def apply(self, layer: LayerObject, x) -> Tensor:
        if not isinstance(x, Tensor):
            raise GenomeError(f"{layer.kind} called on a non-tensor {x!r}")
        layer.calls += 1
        if layer.calls > 1 and layer.kind not in ("Reshape", "MaxPool2D"):
            # shared weights across two call sites: not supported (documented decision)
            raise GenomeError("layer object reused (weight sharing) is not supported")
        cfg = layer.cfg
        k = layer.kind
        if k == "Dense":
            cin = x.shape[-1]
            rows = math.prod(x.shape[:-1])
            return self._add("gemm", [x.node], x.shape[:-1] + (cfg["units"],),
                             dict(kind="dense", rows=1, h=rows, w=1, cin=cin, kh=1, kw=1, sh=1, sw=1,
                                  oh=rows, ow=1, f=cfg["units"], act=cfg["activation"],
                                  use_bias=cfg["use_bias"]))
        if k == "Conv2D":
            if x.ndim < 4:
                raise GenomeError("Conv2D expects min_ndim=4")
            # extra leading batch dims (rank > 4) are unreachable: ranks never exceed 4
            h, w, c = x.shape
            (kh, kw), (sh, sw) = cfg["kernel_size"], cfg["strides"]
            oh, ow = _valid(h, kh, sh), _valid(w, kw, sw)
            return self._add("gemm", [x.node], (oh, ow, cfg["filters"]),
                             dict(kind="conv2d", rows=1, h=h, w=w, cin=c, kh=kh, kw=kw, sh=sh, sw=sw,
                                  oh=oh, ow=ow, f=cfg["filters"], act=cfg["activation"],
                                  use_bias=cfg["use_bias"]))
        if k == "Conv1D":
            if x.ndim < 3:
                raise GenomeError("Conv1D expects min_ndim=3")
            (kk,), (ss,) = cfg["kernel_size"], cfg["strides"]
            c = x.shape[-1]
            if x.ndim == 3:            # (L, C): conv along L
                (l,) = x.shape[:-1]
                ol = _valid(l, kk, ss)
                return self._add("gemm", [x.node], (ol, cfg["filters"]),
                                 dict(kind="conv1d", rows=1, h=l, w=1, cin=c, kh=kk, kw=1, sh=ss, sw=1,
                                      oh=ol, ow=1, f=cfg["filters"], act=cfg["activation"],
                                      use_bias=cfg["use_bias"]))
            # rank-4 input: leading (B, H) are batch dims, convolve along W (TF>=2.5 batch_dims)
            h, w = x.shape[:-1]
            ow = _valid(w, kk, ss)
            return self._add("gemm", [x.node], (h, ow, cfg["filters"]),
                             dict(kind="conv1d", rows=1, h=h, w=w, cin=c, kh=1, kw=kk, sh=1, sw=ss,
                                  oh=h, ow=ow, f=cfg["filters"], act=cfg["activation"],
                                  use_bias=cfg["use_bias"]))
        if k == "MaxPool2D":
            if x.ndim != 4:
                raise GenomeError("MaxPool2D expects ndim=4")
            h, w, c = x.shape
            (ph, pw), (sh, sw) = cfg["pool_size"], cfg["strides"]
            oh, ow = _valid(h, ph, sh), _valid(w, pw, sw)
            return self._add("pool", [x.node], (oh, ow, c),
                             dict(h=h, w=w, c=c, ph=ph, pw=pw, sh=sh, sw=sw, oh=oh, ow=ow))
        if k == "BatchNormalization":
            axis = cfg["axis"]
            nd = x.ndim
            if not _is_int(axis):
                raise GenomeError("BatchNormalization axis must be an int")
            if not -nd <= axis < nd:
                raise GenomeError("BatchNormalization axis out of range")
            ax = axis % nd
            if ax == 0:
                raise GenomeError("BatchNormalization over the batch axis: undefined batch dimension")
            c = x.shape[ax - 1]
            return self._add("bn", [x.node], x.shape,
                             dict(axis=ax, channels=c, momentum=cfg["momentum"], epsilon=cfg["epsilon"],
                                  center=cfg["center"], scale=cfg["scale"],
                                  last=(ax == nd - 1)))
        if k == "Reshape":
            return self._reshape(x, cfg["target_shape"])
        raise GenomeError(f"unknown layer {k}")

    def _reshape(self, x: Tensor, target) -> Tensor:
        original = math.prod(x.shape)
        out = list(target)
        unknown, known = None, 1
        for i, d in enumerate(out):
            if d < 0:
                if unknown is None:
                    unknown = i
                else:
                    raise GenomeError("Can only specify one unknown dimension.")
            else:
                known *= d
        if unknown is not None:
            if known == 0 or original % known != 0:
                raise GenomeError("total size of new array must be unchanged")
            out[unknown] = original // known
        elif original != known:
            raise GenomeError("total size of new array must be unchanged")
        return self._add("reshape", [x.node], tuple(out), {})

    def concatenate(self, tensors: Sequence, axis: int) -> Tensor:
        if not isinstance(tensors, (list, tuple)) or len(tensors) < 1:
            raise GenomeError("A Concatenate layer should be called on a list of at least 1 input")
        if not all(isinstance(t, Tensor) for t in tensors):
            raise GenomeError("Concatenate inputs must be tensors")
        if not _is_int(axis):
            raise GenomeError("concatenate axis must be an int")
        ranks = {t.ndim for t in tensors}
        if len(ranks) != 1:
            raise GenomeError("Concatenate requires inputs with matching ranks")
        nd = ranks.pop()
        if not -nd <= axis < nd:
            raise GenomeError("concatenate axis out of range")
        ax = axis % nd
        if ax == 0:
            raise GenomeError("concatenation over the batch axis is not supported")
        reduced = {tuple(d for i, d in enumerate(t.shape) if i != ax - 1) for t in tensors}
        if len(reduced) != 1:
            raise GenomeError("Concatenate requires matching shapes except for the concat axis")
        shape = list(tensors[0].shape)
        shape[ax - 1] = sum(t.shape[ax - 1] for t in tensors)
        if len(tensors) == 1:
            return tensors[0]
        return self._add("concat", [t.node for t in tensors], tuple(shape), {"axis": ax})

    def neg(self, x: Tensor) -> Tensor:
        return self._add("neg", [x.node], x.shape, {})

    def sub(self, a, b) -> Tensor:
        # broadcasting subtraction between tensors and/or python numbers (KerasTensor.__sub__)
        ta, tb = isinstance(a, Tensor), isinstance(b, Tensor)
        if ta and tb:
            shape = _broadcast(a.shape, b.shape)
            return self._add("sub", [a.node, b.node], shape, {"mode": "tt"})
        if ta:
            return self._add("sub", [a.node], a.shape, {"mode": "tc", "c": float(_num(b))})
        return self._add("sub", [b.node], b.shape, {"mode": "ct", "c": float(_num(a))})


def _num(v):
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v
    if isinstance(v, bool):
        return int(v)
    raise GenomeError(f"unsupported operand {v!r}")


def _broadcast(a: Tuple[int, ...], b: Tuple[int, ...]) -> Tuple[int, ...]:
    """Broadcast two tensor shapes (batch excluded).  Operands of different rank would align a
    concrete dimension with the batch dimension, which only fails at training time in the
    reference (the whole job then crashes); such organisms are reported invalid here."""
    if len(a) != len(b):
        raise GenomeError("operands could not be broadcast together (rank mismatch)")
    out = []
    for da, db in zip(a, b):
        if da == db or db == 1:
            out.append(da)
        elif da == 1:
            out.append(db)
        else:
            raise GenomeError("operands could not be broadcast together")
    return tuple(out)


def _valid(size: int, k: int, s: int) -> int:
    n = size - k + 1
    if n <= 0:
        raise GenomeError(f"negative or zero output size ({size} - {k} + 1)")
    return (n + s - 1) // s


class _Interpreter:
    def __init__(self, builder: _Builder):
        self.b = builder
        self.env: Dict[str, Any] = {
            "Dense": LayerFactory("Dense"),
            "Conv2D": LayerFactory("Conv2D"),
            "Conv1D": LayerFactory("Conv1D"),
            "MaxPool2D": LayerFactory("MaxPool2D"),
            "BatchNormalization": LayerFactory("BatchNormalization"),
            "Reshape": LayerFactory("Reshape"),
            "concatenate": ConcatenateFn(),
            "X_layer": builder.x,
            "g_layer": builder.g,
        }

    # -- statements ------------------------------------------------------------------------------
    def run(self, module: ast.Module):
        for stmt in module.body:
            if isinstance(stmt, ast.Assign):
                value = self.eval(stmt.value)
                for tgt in stmt.targets:
                    self.assign(tgt, value)
            elif isinstance(stmt, ast.Expr):
                self.eval(stmt.value)
            else:
                raise GenomeError(f"unsupported statement {type(stmt).__name__}")

    def assign(self, tgt, value):
        if isinstance(tgt, ast.Name):
            self.env[tgt.id] = value
        elif isinstance(tgt, (ast.Tuple, ast.List)):
            if not isinstance(value, (tuple, list)):
                raise GenomeError("cannot unpack non-sequence")
            if len(value) != len(tgt.elts):
                raise GenomeError("unpack length mismatch")
            for t, v in zip(tgt.elts, value):
                self.assign(t, v)
        else:
            raise GenomeError(f"unsupported assignment target {type(tgt).__name__}")

    # -- expressions -----------------------------------------------------------------------------
    def eval(self, e):
        if isinstance(e, ast.Constant):
            if isinstance(e.value, (int, float, str, bool)) or e.value is None:
                return e.value
            raise GenomeError("unsupported constant")
        if isinstance(e, ast.Name):
            if e.id not in self.env:
                raise GenomeError(f"name {e.id!r} is not defined")
            return self.env[e.id]
        if isinstance(e, ast.Tuple):
            return tuple(self.eval(x) for x in e.elts)
        if isinstance(e, ast.List):
            return [self.eval(x) for x in e.elts]
        if isinstance(e, ast.UnaryOp) and isinstance(e.op, ast.USub):
            v = self.eval(e.operand)
            if isinstance(v, Tensor):
                return self.b.neg(v)
            if isinstance(v, (int, float)):
                return -v
            raise GenomeError("bad operand type for unary -")
        if isinstance(e, ast.BinOp) and isinstance(e.op, ast.Sub):
            a, b = self.eval(e.left), self.eval(e.right)
            if isinstance(a, Tensor) or isinstance(b, Tensor):
                return self.b.sub(a, b)
            if isinstance(a, (int, float)) and isinstance(b, (int, float)):
                return a - b
            raise GenomeError("unsupported operand types for -")
        if isinstance(e, ast.Compare):
            left = self.eval(e.left)
            result = True
            for op, comp in zip(e.ops, e.comparators):
                right = self.eval(comp)
                if isinstance(op, ast.Eq):
                    r = _py_eq(left, right)
                elif isinstance(op, ast.NotEq):
                    r = not _py_eq(left, right)
                else:
                    raise GenomeError("unsupported comparison")
                result = result and r
                left = right
            return result
        if isinstance(e, ast.Call):
            return self.call(e)
        raise GenomeError(f"unsupported expression {type(e).__name__}")

    def call(self, e: ast.Call):
        fn = self.eval(e.func)
        if any(isinstance(a, ast.Starred) for a in e.args) or any(k.arg is None for k in e.keywords):
            raise GenomeError("star-args are not supported")
        args = [self.eval(a) for a in e.args]
        kwargs = {k.arg: self.eval(k.value) for k in e.keywords}
        if isinstance(fn, LayerFactory):
            return LayerObject(fn.kind, _layer_config(fn.kind, args, kwargs))
        if isinstance(fn, LayerObject):
            if kwargs or len(args) != 1:
                raise GenomeError("layer call takes exactly one input")
            return self.b.apply(fn, args[0])
        if isinstance(fn, ConcatenateFn):
            if len(args) < 1 and "inputs" not in kwargs:
                raise GenomeError("concatenate() missing inputs")
            if len(args) > 2:
                raise GenomeError("concatenate() takes at most 2 positional arguments")
            inputs = args[0] if args else kwargs.pop("inputs")
            axis = args[1] if len(args) == 2 else -1
            if "axis" in kwargs:
                if len(args) == 2:
                    raise GenomeError("multiple values for axis")
                axis = kwargs.pop("axis")
            if set(kwargs) - _ALLOWED_BASE_KW:
                raise GenomeError("Keyword argument not understood")
            return self.b.concatenate(inputs, axis)
        raise GenomeError(f"{fn!r} is not callable")


def _py_eq(a, b) -> bool:
    if isinstance(a, (Tensor, LayerObject, LayerFactory, ConcatenateFn)) or \
            isinstance(b, (Tensor, LayerObject, LayerFactory, ConcatenateFn)):
        return a is b
    return a == b


def _layer_config(kind: str, args: list, kwargs: dict) -> Dict[str, Any]:
    sig = _SIGNATURES[kind]
    if len(args) > len(sig):
        raise GenomeError(f"{kind}: unsupported positional argument")
    cfg: Dict[str, Any] = dict(_DEFAULTS[kind])
    given = {}
    for name, val in zip(sig, args):
        given[name] = val
    for k, v in kwargs.items():
        if k in given:
            raise GenomeError(f"{kind}: multiple values for {k}")
        if k not in _KWARGS[kind] and k not in _ALLOWED_BASE_KW:
            raise GenomeError(f"{kind}: Keyword argument not understood: {k}")
        if k not in sig and k not in ("activation", "use_bias") and k not in _DEFAULTS[kind]:
            # accepted by Keras but only meaningful with values the vocabulary cannot express
            raise GenomeError(f"{kind}: unsupported keyword {k}")
        given[k] = v
    for r in _REQUIRED.get(kind, []):
        if r not in given:
            raise GenomeError(f"{kind}: missing required argument {r}")
    cfg.update(given)

    if kind == "Dense":
        cfg["units"] = _to_int(cfg["units"], "units")
        if cfg["units"] <= 0:
            raise GenomeError("units must be positive")
        cfg["activation"] = _activation(cfg["activation"])
        cfg["use_bias"] = bool(cfg["use_bias"])
    elif kind in ("Conv2D", "Conv1D"):
        n = 2 if kind == "Conv2D" else 1
        cfg["filters"] = _to_int(cfg["filters"], "filters")
        if cfg["filters"] <= 0:
            raise GenomeError("filters must be positive")
        cfg["kernel_size"] = _normalize_tuple(cfg["kernel_size"], n, "kernel_size")
        cfg["strides"] = _normalize_tuple(cfg["strides"], n, "strides")
        if min(cfg["kernel_size"]) <= 0 or min(cfg["strides"]) <= 0:
            raise GenomeError("kernel_size and strides must be positive")
        cfg["activation"] = _activation(cfg["activation"])
        cfg["use_bias"] = bool(cfg["use_bias"])
    elif kind == "MaxPool2D":
        cfg["pool_size"] = _normalize_tuple(cfg["pool_size"], 2, "pool_size")
        cfg["strides"] = cfg["pool_size"] if cfg["strides"] is None else \
            _normalize_tuple(cfg["strides"], 2, "strides")
        if min(cfg["pool_size"]) <= 0 or min(cfg["strides"]) <= 0:
            raise GenomeError("pool_size and strides must be positive")
    elif kind == "BatchNormalization":
        cfg["momentum"] = _to_float(cfg["momentum"], "momentum")
        cfg["epsilon"] = _to_float(cfg["epsilon"], "epsilon")
        cfg["center"] = bool(cfg["center"])
        cfg["scale"] = bool(cfg["scale"])
    elif kind == "Reshape":
        ts = cfg["target_shape"]
        if not isinstance(ts, (tuple, list)):
            raise GenomeError("Reshape target_shape must be a tuple")
        if not all(_is_int(d) for d in ts):
            raise GenomeError("Reshape target_shape must contain integers")
        cfg["target_shape"] = tuple(ts)
    return cfg


# ------------------------------------------------------------------------------------------------
# public API
# ------------------------------------------------------------------------------------------------
@dataclass
class InterpretResult:
    ok: bool
    ir: Optional[OrganismIR]
    error: Optional[str]
    parameters_count: float          # NaN when invalid
    loss_balance: float              # NaN when invalid


def interpret(source_code: str, image_shape=(28, 28), genotype_size: int = 100,
              num_classes: int = 10) -> OrganismIR:
    """Interpret ``source_code``; raises :class:`GenomeError` when the reference would fail."""
    if not isinstance(source_code, str):
        raise GenomeError("source code is not a string")
    try:
        module = ast.parse(source_code)
    except (SyntaxError, ValueError) as e:       # ValueError: null bytes
        raise GenomeError(f"SyntaxError: {e}")
    b = _Builder(tuple(image_shape), genotype_size)
    interp = _Interpreter(b)
    try:
        interp.run(module)
    except RecursionError as e:
        raise GenomeError(str(e))
    env = interp.env
    if "con" not in env:
        raise GenomeError("'con' is not defined")
    con = env["con"]
    if not isinstance(con, Tensor):
        raise GenomeError("'con' is not a tensor")
    if "loss_balance" not in env:
        raise GenomeError("'loss_balance' is not defined")
    lb = env["loss_balance"]
    if isinstance(lb, (Tensor, LayerObject, LayerFactory, ConcatenateFn, tuple, list)) or lb is None:
        raise GenomeError("loss_balance is not a number")
    loss_balance = _to_float(lb, "loss_balance")

    # heads: Dense(C)+softmax and Dense(L)+sigmoid on Reshape((1, -1))(con)
    d = math.prod(con.shape)
    flat = b._add("reshape", [con.node], (1, d), {"head": True})
    cls = b._add("gemm", [flat.node], (1, num_classes),
                 dict(kind="head_cls", rows=1, h=1, w=1, cin=d, kh=1, kw=1, sh=1, sw=1, oh=1, ow=1,
                      f=num_classes, act="linear", use_bias=True))
    rep = b._add("gemm", [flat.node], (1, genotype_size),
                 dict(kind="head_rep", rows=1, h=1, w=1, cin=d, kh=1, kw=1, sh=1, sw=1, oh=1, ow=1,
                      f=genotype_size, act="linear", use_bias=True))

    # keep only nodes reachable (backwards) from the heads; inputs are always kept
    keep = {b.x.node, b.g.node}
    stack = [cls.node, rep.node]
    while stack:
        i = stack.pop()
        if i in keep and i not in (b.x.node, b.g.node):
            continue
        keep.add(i)
        stack.extend(b.nodes[i].inputs)
    nodes = [n for n in b.nodes if n.id in keep]
    org = OrganismIR(nodes=nodes, con=con.node, loss_balance=loss_balance, num_classes=num_classes,
                     genotype_size=genotype_size, head_features=d, cls_head=cls.node, rep_head=rep.node)
    return org


def try_interpret(source_code: str, image_shape=(28, 28), genotype_size: int = 100,
                  num_classes: int = 10) -> InterpretResult:
    try:
        ir = interpret(source_code, image_shape, genotype_size, num_classes)
    except GenomeError as e:
        return InterpretResult(False, None, str(e), float("nan"), float("nan"))
    return InterpretResult(True, ir, None, float(ir.count_params()), ir.loss_balance)


def layer_counts(source_code: str) -> Dict[str, int]:
    """Layer statistics parsed from decoded text (experiment.py:323-329)."""
    return {
        "classification_layers": source_code.count("X_layer="),
        "replication_layers": source_code.count("g_layer="),
        "merged_layers": source_code.count("con="),
    }
