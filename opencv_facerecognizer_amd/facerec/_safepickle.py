"""Non-executing pickle reader for facerec model files.

The reference persists models with ``cPickle.dump`` / ``cPickle.load``
(``src/ocvfacerec/facerec/serialization.py:38-49``); the bundled
``data/individuals.pkl`` is a Python-2 protocol-0 stream that names
``copy_reg._reconstructor``, ``numpy.core.multiarray._reconstruct``,
``numpy.matrixlib.defmatrix.matrix``, ``numpy.ndarray`` and ``numpy.dtype``.

``pickle.load`` would import and call whatever the stream names.  This module
instead *interprets the opcodes symbolically*: GLOBAL/REDUCE/BUILD/NEWOBJ
produce inert ``_Global``/``_Call``/``_Build`` nodes, and a separate
materialiser turns only a fixed whitelist of node shapes into objects
(numpy arrays/matrices/dtypes/scalars built from the raw bytes, and the
facerec model classes built from their ``__dict__`` state).  Nothing named in
the file is imported or called.  Protocols 0-4 opcodes are understood.
"""
from __future__ import annotations

import codecs
import struct

import numpy as np


class UnpicklingError(Exception):
    pass


class _Global:
    __slots__ = ("module", "name")

    def __init__(self, module, name):
        self.module, self.name = module, name

    @property
    def qualname(self):
        return f"{self.module}.{self.name}"

    def __repr__(self):
        return f"<global {self.qualname}>"


class _Call:
    __slots__ = ("func", "args", "state", "items", "sets")

    def __init__(self, func, args):
        self.func, self.args = func, args
        self.state = None
        self.items = None   # list appends (for list subclasses)
        self.sets = None    # dict setitems (for dict subclasses)

    def __repr__(self):
        return f"<call {self.func!r}{self.args!r}>"


class _Mark:
    pass


class _Str8(bytes):
    """A py2 ``str`` (STRING/BINSTRING/SHORT_BINSTRING): text unless consumed as raw bytes."""


_MARK = _Mark()


def _decode_py2_string(raw: bytes) -> bytes:
    """Protocol-0 STRING argument: a quoted repr() of a py2 ``str``."""
    raw = raw.rstrip(b"\r")
    if len(raw) < 2 or raw[0] != raw[-1] or raw[:1] not in (b"'", b'"'):
        raise UnpicklingError("malformed STRING opcode")
    return codecs.escape_decode(raw[1:-1])[0]


def parse(data: bytes):
    """Run the opcode stream into a symbolic object tree (no side effects)."""
    stack = []
    memo = {}
    pos = 0
    n = len(data)

    def readline():
        nonlocal pos
        e = data.find(b"\n", pos)
        if e < 0:
            raise UnpicklingError("truncated line")
        s = data[pos:e]
        pos = e + 1
        return s

    def read(k):
        nonlocal pos
        if pos + k > n:
            raise UnpicklingError("truncated stream")
        s = data[pos:pos + k]
        pos += k
        return s

    def pop_mark():
        items = []
        while True:
            if not stack:
                raise UnpicklingError("mark not found")
            x = stack.pop()
            if x is _MARK:
                break
            items.append(x)
        items.reverse()
        return items

    def add_items(lst, items):
        if isinstance(lst, list):
            lst.extend(items)
        elif isinstance(lst, _Call):
            lst.items = (lst.items or []) + list(items)
        else:
            raise UnpicklingError("APPEND to non-list")

    def set_items(d, kv):
        if isinstance(d, dict):
            for k, v in kv:
                d[_hashable(k)] = v
        elif isinstance(d, _Call):
            d.sets = (d.sets or []) + list(kv)
        else:
            raise UnpicklingError("SETITEM on non-dict")

    while True:
        if pos >= n:
            raise UnpicklingError("no STOP opcode")
        op = data[pos:pos + 1]
        pos += 1
        if op == b".":  # STOP
            if len(stack) != 1:
                raise UnpicklingError("bad stack at STOP")
            return stack[0]
        elif op == b"(":
            stack.append(_MARK)
        elif op == b"0":
            stack.pop()
        elif op == b"1":
            pop_mark()
        elif op == b"2":
            stack.append(stack[-1])
        elif op == b"N":
            stack.append(None)
        elif op == b"\x88":
            stack.append(True)
        elif op == b"\x89":
            stack.append(False)
        elif op == b"I":
            s = readline()
            if s == b"00":
                stack.append(False)
            elif s == b"01":
                stack.append(True)
            else:
                stack.append(int(s))
        elif op == b"L":
            stack.append(int(readline().rstrip(b"L")))
        elif op == b"F":
            stack.append(float(readline()))
        elif op == b"J":
            stack.append(struct.unpack("<i", read(4))[0])
        elif op == b"K":
            stack.append(read(1)[0])
        elif op == b"M":
            stack.append(struct.unpack("<H", read(2))[0])
        elif op == b"G":
            stack.append(struct.unpack(">d", read(8))[0])
        elif op == b"\x8a":
            k = read(1)[0]
            stack.append(int.from_bytes(read(k), "little", signed=True))
        elif op == b"\x8b":
            k = struct.unpack("<i", read(4))[0]
            stack.append(int.from_bytes(read(k), "little", signed=True))
        elif op == b"S":
            stack.append(_Str8(_decode_py2_string(readline())))
        elif op == b"T":
            k = struct.unpack("<i", read(4))[0]
            stack.append(_Str8(read(k)))
        elif op == b"U":
            stack.append(_Str8(read(read(1)[0])))
        elif op == b"B":
            stack.append(read(struct.unpack("<I", read(4))[0]))
        elif op == b"C":
            stack.append(read(read(1)[0]))
        elif op == b"\x8e":
            stack.append(read(struct.unpack("<Q", read(8))[0]))
        elif op == b"\x96":
            stack.append(bytes(read(struct.unpack("<Q", read(8))[0])))
        elif op == b"V":
            stack.append(readline().decode("raw_unicode_escape"))
        elif op == b"X":
            stack.append(read(struct.unpack("<I", read(4))[0]).decode("utf-8", "surrogatepass"))
        elif op == b"\x8c":
            stack.append(read(read(1)[0]).decode("utf-8", "surrogatepass"))
        elif op == b"\x8d":
            stack.append(read(struct.unpack("<Q", read(8))[0]).decode("utf-8", "surrogatepass"))
        elif op == b"]":
            stack.append([])
        elif op == b"l":
            stack.append(pop_mark())
        elif op == b"a":
            v = stack.pop()
            add_items(stack[-1], [v])
        elif op == b"e":
            items = pop_mark()
            add_items(stack[-1], items)
        elif op == b"}":
            stack.append({})
        elif op == b"d":
            items = pop_mark()
            stack.append({_hashable(items[i]): items[i + 1] for i in range(0, len(items), 2)})
        elif op == b"s":
            v = stack.pop()
            k = stack.pop()
            set_items(stack[-1], [(k, v)])
        elif op == b"u":
            items = pop_mark()
            set_items(stack[-1], [(items[i], items[i + 1]) for i in range(0, len(items), 2)])
        elif op == b")":
            stack.append(())
        elif op == b"t":
            stack.append(tuple(pop_mark()))
        elif op == b"\x85":
            stack.append((stack.pop(),))
        elif op == b"\x86":
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b))
        elif op == b"\x87":
            c = stack.pop()
            b = stack.pop()
            a = stack.pop()
            stack.append((a, b, c))
        elif op == b"\x8f":
            stack.append(set())
        elif op == b"\x90":
            items = pop_mark()
            stack[-1].update(_hashable(x) for x in items)
        elif op == b"\x91":
            stack.append(frozenset(_hashable(x) for x in pop_mark()))
        elif op == b"p":
            memo[int(readline())] = stack[-1]
        elif op == b"q":
            memo[read(1)[0]] = stack[-1]
        elif op == b"r":
            memo[struct.unpack("<I", read(4))[0]] = stack[-1]
        elif op == b"\x94":
            memo[len(memo)] = stack[-1]
        elif op == b"g":
            stack.append(memo[int(readline())])
        elif op == b"h":
            stack.append(memo[read(1)[0]])
        elif op == b"j":
            stack.append(memo[struct.unpack("<I", read(4))[0]])
        elif op == b"c":
            module = readline().decode("ascii")
            name = readline().decode("ascii")
            stack.append(_Global(module, name))
        elif op == b"\x93":
            name = stack.pop()
            module = stack.pop()
            stack.append(_Global(module, name))
        elif op == b"R":
            args = stack.pop()
            func = stack.pop()
            stack.append(_Call(func, tuple(args)))
        elif op == b"\x81":
            args = stack.pop()
            cls = stack.pop()
            stack.append(_Call(_Global("__newobj__", "__newobj__"), (cls,) + tuple(args)))
        elif op == b"\x92":
            kwargs = stack.pop()
            args = stack.pop()
            cls = stack.pop()
            if kwargs:
                raise UnpicklingError("NEWOBJ_EX with kwargs is not supported")
            stack.append(_Call(_Global("__newobj__", "__newobj__"), (cls,) + tuple(args)))
        elif op == b"i":
            module = readline().decode("ascii")
            name = readline().decode("ascii")
            args = pop_mark()
            stack.append(_Call(_Global(module, name), tuple(args)))
        elif op == b"o":
            items = pop_mark()
            stack.append(_Call(_Global("__newobj__", "__newobj__"), tuple(items)))
        elif op == b"b":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, _Call):
                raise UnpicklingError("BUILD on a non-reconstructed object")
            obj.state = state
        elif op == b"\x80":
            read(1)
        elif op == b"\x95":
            read(8)
        else:
            raise UnpicklingError(f"unsupported opcode {op!r} at {pos - 1}")


def _hashable(k):
    if isinstance(k, (list, dict, _Call)):
        raise UnpicklingError("unhashable key in pickle")
    return k


# --------------------------------------------------------------------------
# Materialisation (whitelist only)
# --------------------------------------------------------------------------

_NP_RECONSTRUCT = {
    "numpy.core.multiarray._reconstruct",
    "numpy._core.multiarray._reconstruct",
}
_NP_ARRAY_TYPES = {
    "numpy.ndarray": np.ndarray,
    "numpy.matrixlib.defmatrix.matrix": np.matrix,
    "numpy.matrix": np.matrix,
}
_NP_DTYPE = {"numpy.dtype"}
_NP_SCALAR = {"numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar"}
_COPYREG = {"copy_reg._reconstructor", "copyreg._reconstructor"}
_OBJECT = {"__builtin__.object", "builtins.object"}
_BUILTIN_CONTAINERS = {
    "__builtin__.set": set, "builtins.set": set,
    "__builtin__.frozenset": frozenset, "builtins.frozenset": frozenset,
    "__builtin__.list": list, "builtins.list": list,
    "__builtin__.tuple": tuple, "builtins.tuple": tuple,
    "__builtin__.dict": dict, "builtins.dict": dict,
}


def _as_bytes(x):
    if isinstance(x, bytes):
        return bytes(x)
    if isinstance(x, str):  # py2 str read back as text: latin-1 is lossless
        return x.encode("latin-1")
    raise UnpicklingError("expected raw bytes")


def _as_text(x):
    if isinstance(x, bytes):
        return x.decode("latin-1")
    return x


# Derived device state (classifier ``_dev``, feature ``_dev_proj``, PCA ``_shift_cache``) is never
# pickled by this package (``__getstate__`` drops it); a file that carries such keys must not
# pre-seed the caches, whose identity checks would then be bypassed.
def _is_cache_key(k):
    return isinstance(k, str) and (k.startswith("_dev") or k in ("_shift_cache", "_shard"))


def _drop_caches(st):
    if not isinstance(st, dict):
        raise UnpicklingError("instance state must be a dict")
    return {k: v for k, v in st.items() if not _is_cache_key(k)}


class _Materializer:
    def __init__(self, classes):
        self.classes = classes   # qualname -> python class
        self.done = {}           # id(node) -> object

    def __call__(self, node):
        if isinstance(node, (_Call, list, dict, tuple, set, frozenset)):
            key = id(node)
            if key in self.done:
                return self.done[key]
        if isinstance(node, _Call):
            obj = self._call(node)
        elif isinstance(node, list):
            obj = []
            self.done[id(node)] = obj
            obj.extend(self(x) for x in node)
            return obj
        elif isinstance(node, dict):
            obj = {}
            self.done[id(node)] = obj
            for k, v in node.items():
                obj[self(k)] = self(v)
            return obj
        elif isinstance(node, tuple):
            obj = tuple(self(x) for x in node)
        elif isinstance(node, (set, frozenset)):
            obj = type(node)(self(x) for x in node)
        elif isinstance(node, _Global):
            raise UnpicklingError(f"bare global {node.qualname} is not allowed")
        elif isinstance(node, _Str8):
            return bytes(node).decode("latin-1")
        else:
            return node
        if isinstance(node, (_Call, tuple, set, frozenset)):
            self.done[id(node)] = obj
        return obj

    # -- helpers ----------------------------------------------------------
    def _dtype(self, node):
        if not (isinstance(node, _Call) and isinstance(node.func, _Global) and node.func.qualname in _NP_DTYPE):
            raise UnpicklingError("expected numpy.dtype")
        key = id(node)
        if key in self.done:
            return self.done[key]
        code = _as_text(node.args[0])
        dt = np.dtype(code)
        st = node.state
        if st is not None and dt.itemsize > 1 and len(st) > 1 and st[1] in (b">", ">", b"<", "<"):
            dt = dt.newbyteorder(_as_text(st[1]))
        if st is not None and len(st) >= 5 and st[3] not in (None,):
            raise UnpicklingError("structured dtypes are not supported")
        self.done[key] = dt
        return dt

    def _call(self, node):
        f = node.func
        if not isinstance(f, _Global):
            raise UnpicklingError("call of a non-global")
        q = f.qualname
        if q in _NP_RECONSTRUCT:
            return self._ndarray(node)
        if q in _NP_DTYPE:
            return self._dtype(node)
        if q in _NP_SCALAR:
            dt = self._dtype(node.args[0])
            raw = node.args[1]
            raw = _as_bytes(self(raw) if isinstance(raw, _Call) else raw)
            return np.frombuffer(raw, dtype=dt, count=1)[0]
        if q in _COPYREG:
            cls_node, base_node, base_state = node.args
            if not (isinstance(base_node, _Global) and base_node.qualname in _OBJECT) or base_state is not None:
                raise UnpicklingError("only object-based copy_reg reconstruction is allowed")
            return self._instance(cls_node, node)
        if q == "__newobj__.__newobj__":
            cls_node = node.args[0]
            if isinstance(cls_node, _Global) and cls_node.qualname in _BUILTIN_CONTAINERS:
                typ = _BUILTIN_CONTAINERS[cls_node.qualname]
                if typ is list:
                    return [self(x) for x in (node.items or [])]
                if typ is dict:
                    return {self(k): self(v) for k, v in (node.sets or [])}
                return typ(self(x) for x in node.args[1:][0]) if len(node.args) > 1 else typ()
            if len(node.args) > 1:
                raise UnpicklingError("NEWOBJ with arguments is not allowed for model classes")
            return self._instance(cls_node, node)
        if q in ("numpy.core.numeric._frombuffer", "numpy._core.numeric._frombuffer"):
            raw, dt_node, shape, order = node.args
            dt = self._dtype(dt_node)
            if dt.hasobject:
                raise UnpicklingError("object arrays are not allowed")
            buf = _as_bytes(self(raw) if isinstance(raw, _Call) else raw)
            shape = tuple(int(x) for x in shape)
            return np.frombuffer(buf, dtype=dt).copy().reshape(shape, order=_as_text(order))
        if q in ("_codecs.encode", "codecs.encode"):
            # py3 protocol<3 spelling of a bytes literal: encode(text, 'latin1')
            text, enc = node.args[0], _as_text(node.args[1]) if len(node.args) > 1 else "utf-8"
            if not isinstance(text, str) or enc.lower().replace("-", "") not in ("latin1", "latin", "iso88591"):
                raise UnpicklingError("only latin-1 codecs.encode is allowed")
            return text.encode("latin-1")
        if q in ("__builtin__.bytes", "builtins.bytes") and not node.args:
            return b""
        if q in _BUILTIN_CONTAINERS:
            typ = _BUILTIN_CONTAINERS[q]
            return typ(self(node.args[0])) if node.args else typ()
        raise UnpicklingError(f"global {q} is not whitelisted")

    def _instance(self, cls_node, node):
        """Build a whitelisted facerec instance; device-cache slots in the file are ignored."""
        if not isinstance(cls_node, _Global):
            raise UnpicklingError("class must be a global")
        cls = self.classes.get(cls_node.qualname)
        if cls is None:
            raise UnpicklingError(f"class {cls_node.qualname} is not whitelisted")
        obj = cls.__new__(cls)
        self.done[id(node)] = obj
        state = node.state
        if state is not None:
            slotstate = None
            if isinstance(state, tuple) and len(state) == 2:
                state, slotstate = state
            st = self(state) if state is not None else {}
            if not isinstance(st, dict):
                raise UnpicklingError("instance state must be a dict")
            st = _drop_caches(st)
            if hasattr(obj, "__setstate__") and getattr(cls, "_facerec_setstate", False):
                obj.__setstate__(st)
            else:
                obj.__dict__.update(st)
            if slotstate:
                for k, v in _drop_caches(self(slotstate)).items():
                    setattr(obj, k, v)
        return obj

    def _ndarray(self, node):
        sub, shape0, dtype_code = node.args
        if not isinstance(sub, _Global) or sub.qualname not in _NP_ARRAY_TYPES:
            raise UnpicklingError("ndarray subtype is not whitelisted")
        st = node.state
        if st is None:
            raise UnpicklingError("ndarray without state")
        if len(st) == 5:
            _ver, shape, dt_node, is_fortran, raw = st
        elif len(st) == 4:
            shape, dt_node, is_fortran, raw = st
        else:
            raise UnpicklingError("unexpected ndarray state")
        dt = self._dtype(dt_node)
        if dt.hasobject:
            raise UnpicklingError("object arrays are not allowed")
        shape = tuple(int(s) for s in shape)
        count = int(np.prod(shape)) if shape else 1
        if isinstance(raw, list):
            raise UnpicklingError("object arrays are not allowed")
        buf = _as_bytes(self(raw) if isinstance(raw, _Call) else raw)
        if len(buf) != count * dt.itemsize:
            raise UnpicklingError("ndarray byte count mismatch")
        arr = np.frombuffer(buf, dtype=dt, count=count).copy()
        arr = arr.reshape(shape, order="F" if is_fortran else "C")
        if dt.byteorder == ">":
            arr = arr.astype(dt.newbyteorder("="))
        typ = _NP_ARRAY_TYPES[sub.qualname]
        if typ is np.matrix:
            arr = np.asmatrix(arr)
        return arr


def loads(data: bytes, classes: dict):
    """Parse ``data`` and build objects using only ``classes`` (qualname -> cls)."""
    tree = parse(data)
    return _Materializer(classes)(tree)
