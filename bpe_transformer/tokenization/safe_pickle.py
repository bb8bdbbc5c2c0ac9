"""A pickle READER that constructs only builtin data: ints, bytes, str, lists, tuples, dicts and sets.

Tokenizer artifacts (``vocab.pkl`` = ``dict[int, bytes]``, ``merges.pkl`` = ``list[tuple[bytes, bytes]]``,
reference ``bpe_trainer.py:447-472``) are pickles, and files of that format may come from anywhere.  This module
never calls ``pickle.load`` or any ``Unpickler``: it walks the opcode stream with :func:`pickletools.genops`
(a parser; it constructs nothing) and interprets the handful of opcodes such containers use on a private
stack.  Every opcode that could look up a global, call a callable or build an object (``GLOBAL``,
``STACK_GLOBAL``, ``REDUCE``, ``BUILD``, ``INST``, ``OBJ``, ``NEWOBJ``, extension codes, persistent ids ...)
raises :class:`UnsafePickleError`, so nothing from the file is ever executed.

Covers protocols 2-5 as written by ``pickle.dump`` for these types (``MEMOIZE`` / ``BINPUT`` memo,
``FRAME``, ``SHORT_BINBYTES`` ... ``BINBYTES8``, ``SETITEMS``, ``APPENDS``, ``TUPLE2``, and the set opcodes
``EMPTY_SET`` / ``ADDITEMS`` / ``FROZENSET`` of the reference's snapshot pickles).
"""

from __future__ import annotations

import pickletools


class UnsafePickleError(ValueError):
    """The pickle uses an opcode outside the builtin-data subset."""


_TUPLE_N = {"TUPLE1": 1, "TUPLE2": 2, "TUPLE3": 3}
_SCALARS = {
    "BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG",
    "SHORT_BINBYTES", "BINBYTES", "BINBYTES8",
    "SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE",
    "BINFLOAT", "FLOAT",
}


def loads(data: bytes):
    """Decode a pickle of builtin containers of ints / bytes / str / floats; raise on anything else.

    Every failure -- a refused opcode, or a malformed / hostile stream (GET before PUT, an empty stack or mark
    stack, an unhashable dict key, SETITEM on a list, a truncated opcode) -- raises :class:`UnsafePickleError`."""
    try:
        return _loads(data)
    except UnsafePickleError:
        raise
    except (KeyError, IndexError, TypeError, AttributeError, ValueError, EOFError) as e:
        raise UnsafePickleError(f"malformed pickle ({type(e).__name__}: {e})") from None


def _loads(data: bytes):
    stack: list = []
    marks: list[int] = []
    memo: dict[int, object] = {}
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name in _SCALARS:
            if name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
                stack.append(bytes(arg))
            else:
                stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name in ("NEWTRUE", "NEWFALSE"):
            stack.append(name == "NEWTRUE")
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "EMPTY_SET":
            stack.append(set())
        elif name == "ADDITEMS":
            k0 = marks.pop()
            items = stack[k0:]
            del stack[k0:]
            if not isinstance(stack[-1], set):
                raise UnsafePickleError("malformed pickle: ADDITEMS on a non-set")
            stack[-1].update(items)
        elif name == "FROZENSET":
            k0 = marks.pop()
            items = stack[k0:]
            del stack[k0:]
            stack.append(frozenset(items))
        elif name == "MARK":
            marks.append(len(stack))
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            k0 = marks.pop()
            items = stack[k0:]
            del stack[k0:]
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            k0 = marks.pop()
            items = stack[k0:]
            del stack[k0:]
            stack[-1].extend(items)
        elif name in _TUPLE_N:
            n = _TUPLE_N[name]
            if len(stack) < n:
                raise UnsafePickleError(f"malformed pickle: {name} on a stack of {len(stack)}")
            t = tuple(stack[-n:])
            del stack[-n:]
            stack.append(t)
        elif name in ("TUPLE", "LIST", "DICT"):
            k0 = marks.pop()
            items = stack[k0:]
            del stack[k0:]
            if name == "TUPLE":
                stack.append(tuple(items))
            elif name == "LIST":
                stack.append(list(items))
            else:
                stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif name == "STOP":
            if len(stack) != 1:
                raise UnsafePickleError("malformed pickle: stack not empty at STOP")
            return stack.pop()
        else:
            raise UnsafePickleError(f"refusing pickle opcode {name} (only builtin data is accepted)")
    raise UnsafePickleError("malformed pickle: no STOP opcode")


def load(path) -> object:
    with open(path, "rb") as f:
        return loads(f.read())
