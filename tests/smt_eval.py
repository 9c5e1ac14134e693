"""Test-only evaluation of expression DAGs under a model (z3 model.eval with
model_completion=True, support_utils.py:65): the third, pure-Python restatement
next to the C oracle (oracle/bv_ref.c) and the device (bv_eval.cuh).

It evaluates the DAG as built (arrays as store chains over K / symbolic arrays,
uninterpreted-function applications, values of any width), not the lowered
256-bit program, so it checks the lowering too.  Models: var name -> int,
array name -> ArrayInterp, function name -> FuncInterp; anything absent is
completed with 0."""
from mythril_amd.smt.program import ArrayInterp, FuncInterp
from mythril_amd.smt.semantics import apply_op


def _m(w):
    return (1 << w) - 1


def evaluate(node, model: dict, cache=None):
    cache = {} if cache is None else cache
    stack = [(node, False)]
    while stack:
        n, ready = stack.pop()
        if n in cache:
            continue
        if n.op == "const":
            cache[n] = n.param
            continue
        if n.op == "var":
            v = model.get(n.param, 0)
            cache[n] = (v if isinstance(v, int) else 0) & _m(n.width)
            continue
        if n.op == "array":
            interp = model.get(n.param[0])
            if isinstance(interp, ArrayInterp):
                cache[n] = (interp.default, dict(interp.entries))
            else:
                cache[n] = (0, {})
            continue
        if not ready:
            stack.append((n, True))
            for c in n.args:
                if c not in cache:
                    stack.append((c, False))
            continue
        vals = [cache[c] for c in n.args]
        if n.op == "K":
            cache[n] = (vals[0], {})
        elif n.op == "store":
            default, entries = vals[0]
            e = dict(entries)
            e[vals[1]] = vals[2]
            cache[n] = (default, e)
        elif n.op == "select":
            default, entries = vals[0]
            cache[n] = entries.get(vals[1], default)
        elif n.op == "uf":
            interp = model.get(n.param[0])
            if isinstance(interp, FuncInterp):
                cache[n] = interp.entries.get(tuple(vals), interp.else_value) & _m(n.width)
            else:
                cache[n] = 0
        else:
            cache[n] = apply_op(n.op, n.width, vals, [c.width for c in n.args], n.param)
    return cache[node]
