"""Test-only evaluation of expression DAGs under a model (z3 model.eval with
model_completion=True, support_utils.py:65): the third, pure-Python restatement
next to the C oracle (oracle/bv_ref.c) and the device (bv_eval.cuh)."""
from mythril_amd.smt.semantics import apply_op


def _m(w):
    return (1 << w) - 1


def evaluate(node, model: dict, cache=None) -> int:
    """Value of an expression DAG under `model` (var name -> int); variables absent
    from the model take 0 (z3 model_completion, support_utils.py:65)."""
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
            cache[n] = model.get(n.param, 0) & _m(n.width)
            continue
        if not ready:
            stack.append((n, True))
            for c in n.args:
                if c not in cache:
                    stack.append((c, False))
            continue
        cache[n] = apply_op(n.op, n.width, [cache[c] for c in n.args], [c.width for c in n.args],
                            n.param)
    return cache[node]
