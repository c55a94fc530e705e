"""A data-only pickle reader that never executes anything from the file.

The reference stores its shard metadata as pickles (``bert_nid2index.pkl``,
``train_sam_uid.pkl``, ``valid_sam_uid.pkl``; read with ``pickle5.load`` at
``client.py:229-240``).  Loading such a file with :mod:`pickle` can run arbitrary code,
so this module interprets the pickle *opcode stream* itself and only understands the
opcodes that build plain data: ``dict``/``list``/``tuple``/``set``/``str``/``bytes``/
``int``/``float``/``bool``/``None``.  Any opcode that would look up a global or call
something (``GLOBAL``, ``STACK_GLOBAL``, ``REDUCE``, ``BUILD``, ``NEWOBJ``, ``INST``,
``OBJ``, ``EXT*``, ``PERSID`` ...) raises :class:`UnsafePickleError`.

Writing uses the standard :func:`pickle.dump` (protocol 4), which produces exactly the
opcodes this reader accepts for such data.
"""
from __future__ import annotations

import io
import pickle
import struct
from typing import Any, BinaryIO, List


class UnsafePickleError(ValueError):
    pass


_MARK = object()


def _read_exact(f: BinaryIO, n: int) -> bytes:
    b = f.read(n)
    if len(b) != n:
        raise EOFError("truncated pickle")
    return b


def _decode_long(b: bytes) -> int:
    return int.from_bytes(b, "little", signed=True) if b else 0


def loads(data: bytes) -> Any:
    return load(io.BytesIO(data))


def load_path(path) -> Any:
    with open(path, "rb") as f:
        return load(f)


def load(f: BinaryIO) -> Any:  # noqa: C901 - a flat opcode switch reads best
    stack: List[Any] = []
    memo: dict = {}

    def pop_mark() -> List[Any]:
        for i in range(len(stack) - 1, -1, -1):
            if stack[i] is _MARK:
                items = stack[i + 1:]
                del stack[i:]
                return items
        raise UnsafePickleError("MARK not found")

    while True:
        op = f.read(1)
        if not op:
            raise EOFError("pickle ended without STOP")
        c = op[0]
        if c == 0x80:  # PROTO
            _read_exact(f, 1)
        elif c == 0x95:  # FRAME
            _read_exact(f, 8)
        elif c == 0x2E:  # STOP
            if len(stack) != 1:
                raise UnsafePickleError("malformed stack at STOP")
            return stack.pop()
        elif c == 0x28:  # MARK
            stack.append(_MARK)
        elif c == 0x7D:  # EMPTY_DICT
            stack.append({})
        elif c == 0x5D:  # EMPTY_LIST
            stack.append([])
        elif c == 0x29:  # EMPTY_TUPLE
            stack.append(())
        elif c == 0x8F:  # EMPTY_SET
            stack.append(set())
        elif c == 0x4E:  # NONE
            stack.append(None)
        elif c == 0x88:  # NEWTRUE
            stack.append(True)
        elif c == 0x89:  # NEWFALSE
            stack.append(False)
        elif c == 0x4B:  # BININT1
            stack.append(_read_exact(f, 1)[0])
        elif c == 0x4D:  # BININT2
            stack.append(struct.unpack("<H", _read_exact(f, 2))[0])
        elif c == 0x4A:  # BININT
            stack.append(struct.unpack("<i", _read_exact(f, 4))[0])
        elif c == 0x8A:  # LONG1
            n = _read_exact(f, 1)[0]
            stack.append(_decode_long(_read_exact(f, n)))
        elif c == 0x8B:  # LONG4
            n = struct.unpack("<i", _read_exact(f, 4))[0]
            if n < 0 or n > (1 << 20):
                raise UnsafePickleError("LONG4 length out of range")
            stack.append(_decode_long(_read_exact(f, n)))
        elif c == 0x47:  # BINFLOAT
            stack.append(struct.unpack(">d", _read_exact(f, 8))[0])
        elif c == 0x8C:  # SHORT_BINUNICODE
            n = _read_exact(f, 1)[0]
            stack.append(_read_exact(f, n).decode("utf-8", "surrogatepass"))
        elif c == 0x58:  # BINUNICODE
            n = struct.unpack("<I", _read_exact(f, 4))[0]
            stack.append(_read_exact(f, n).decode("utf-8", "surrogatepass"))
        elif c == 0x8D:  # BINUNICODE8
            n = struct.unpack("<Q", _read_exact(f, 8))[0]
            stack.append(_read_exact(f, n).decode("utf-8", "surrogatepass"))
        elif c == 0x43:  # SHORT_BINBYTES
            n = _read_exact(f, 1)[0]
            stack.append(_read_exact(f, n))
        elif c == 0x42:  # BINBYTES
            n = struct.unpack("<I", _read_exact(f, 4))[0]
            stack.append(_read_exact(f, n))
        elif c == 0x94:  # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif c == 0x71:  # BINPUT
            memo[_read_exact(f, 1)[0]] = stack[-1]
        elif c == 0x72:  # LONG_BINPUT
            memo[struct.unpack("<I", _read_exact(f, 4))[0]] = stack[-1]
        elif c == 0x68:  # BINGET
            stack.append(memo[_read_exact(f, 1)[0]])
        elif c == 0x6A:  # LONG_BINGET
            stack.append(memo[struct.unpack("<I", _read_exact(f, 4))[0]])
        elif c == 0x61:  # APPEND
            v = stack.pop()
            stack[-1].append(v)
        elif c == 0x65:  # APPENDS
            items = pop_mark()
            stack[-1].extend(items)
        elif c == 0x73:  # SETITEM
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif c == 0x75:  # SETITEMS
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif c == 0x90:  # ADDITEMS
            items = pop_mark()
            stack[-1].update(items)
        elif c == 0x91:  # FROZENSET
            stack.append(frozenset(pop_mark()))
        elif c == 0x74:  # TUPLE
            stack.append(tuple(pop_mark()))
        elif c == 0x85:  # TUPLE1
            stack[-1:] = [(stack[-1],)]
        elif c == 0x86:  # TUPLE2
            stack[-2:] = [tuple(stack[-2:])]
        elif c == 0x87:  # TUPLE3
            stack[-3:] = [tuple(stack[-3:])]
        elif c == 0x6C:  # LIST
            stack.append(list(pop_mark()))
        elif c == 0x64:  # DICT
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif c == 0x30:  # POP
            stack.pop()
        elif c == 0x31:  # POP_MARK
            pop_mark()
        elif c == 0x32:  # DUP
            stack.append(stack[-1])
        else:
            raise UnsafePickleError(
                f"opcode 0x{c:02x} is not a plain-data opcode; refusing to interpret it"
            )


def dump_path(obj: Any, path) -> None:
    with open(path, "wb") as f:
        pickle.dump(obj, f, protocol=4)
