"""Extract the reference's golden regression outputs (``/root/reference/tests/expected.pkl``,
consumed by ``tests/test_model.py:143-189`` upstream) into ``expected_outputs.json``.

The file is a Python pickle.  It is NOT unpickled: no ``pickle.load``/``torch.load`` runs on it.
Instead the opcode stream is walked with ``pickletools.genops`` (a pure disassembler that executes
nothing) by a tiny stack machine that understands only containers, scalars and the
``torch._utils._rebuild_tensor_v2(torch.storage._load_from_bytes(<bytes>), offset, size, stride, ...)``
pattern.  The nested storage blob (legacy ``torch.save`` format) is parsed the same way and its
raw little-endian float32/float64 payload read with numpy.  Globals are recorded by NAME only and
never resolved.  Run in this container only (needs /root/reference); the JSON is the fixture.
"""
import io
import json
import os
import pickletools
import sys

import numpy as np

SRC = "/root/reference/tests/expected.pkl"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expected_outputs.json")

_DTYPES = {"FloatStorage": np.float32, "DoubleStorage": np.float64, "LongStorage": np.int64}


class Global:
    def __init__(self, module, name):
        self.qual = f"{module}.{name}"


class Call:
    def __init__(self, fn, args):
        self.fn, self.args = fn, args


def _storage_from_legacy_blob(blob):
    f = io.BytesIO(blob)
    storage_type = None
    for _ in range(5):  # magic, protocol, sys_info, storage record, key list
        for op, arg, _pos in pickletools.genops(f):
            if op.name == "GLOBAL":
                storage_type = arg.split(" ")[1]
            if op.name == "STOP":
                break
    count = int(np.frombuffer(f.read(8), dtype="<i8")[0])
    dt = _DTYPES[storage_type]
    return np.frombuffer(f.read(count * np.dtype(dt).itemsize), dtype=dt).copy()


def _materialize(obj):
    if isinstance(obj, Call):
        if obj.fn.qual == "torch._utils._rebuild_tensor_v2":
            storage, offset, size, stride = obj.args[:4]
            storage = _materialize(storage)
            arr = np.lib.stride_tricks.as_strided(
                storage[offset:], shape=size, strides=[s * storage.itemsize for s in stride])
            return np.array(arr)
        if obj.fn.qual == "torch.storage._load_from_bytes":
            return _storage_from_legacy_blob(obj.args[0])
        if obj.fn.qual == "collections.OrderedDict":
            return {}
        raise ValueError(f"refusing to interpret global {obj.fn.qual}")
    if isinstance(obj, dict):
        return {k: _materialize(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_materialize(v) for v in obj)
    return obj


def walk(data):
    stack, memo, marks = [], {}, []
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        elif n == "STOP":
            break
        elif n == "MARK":
            marks.append(len(stack))
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BININT1", "BININT2", "BININT", "BINBYTES",
                   "SHORT_BINBYTES", "BINFLOAT", "LONG1"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "TUPLE":
            m = marks.pop()
            items = tuple(stack[m:])
            del stack[m:]
            stack.append(items)
        elif n == "SETITEMS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(Global(module, name))
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(Call(fn, args))
        else:
            raise ValueError(f"unsupported opcode {n}")
    return _materialize(stack[-1])


def main():
    tree = walk(open(SRC, "rb").read())
    out = {}
    for model, per_out in tree.items():
        out[model] = {}
        for head, vals in per_out.items():
            out[model][head] = {k: (None if v is None else {"shape": list(v.shape), "values": v.ravel().tolist()})
                                for k, v in vals.items()}
    json.dump(out, open(OUT, "w"), indent=1)
    for model, per_out in out.items():
        for head, vals in per_out.items():
            print(model, head, vals["pred"]["values"][:4])


if __name__ == "__main__":
    sys.exit(main())
