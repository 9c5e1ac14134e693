"""Refutation under the keccak axioms -- the part of an SMT solver's answer the
SAT-only backend (search.py) can give without one.

A mapping read in a fresh contract, ``select(store(K(0), 0, v), keccak256_512(
sender . 1))``, is 0 in every model of a query that carries the keccak
conditions (keccak_function_manager.py:116-179): the application lies in its
size's interval [lo, lo + PART) on a multiple of 64, or equals a registered
concrete hash of the same size -- never the constant slot 0.  z3 proves such a
path unsat and the reference prunes it (constraints.py:35-38); a search over
candidate models can only fail to find one ("unknown"), keeping the path alive
and every query below it.  ``refutes(conjuncts)`` rewrites each conjunct with
that one axiom -- a store at a constant key the application provably differs
from is skipped, a constant array answers its default -- folds constants back
up, and reports a conjunct that becomes False.  Sound: the rewrite is applied
only to applications whose keccak condition is itself a conjunct of the query,
and only the exact intervals/concrete hashes the condition states are used.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Set

from .expr import FALSE, Node, _fold


def _keccak_facts(conj: Set[Node]):
    """{keccak application node: (lo, hi, concrete hash values of its size)}
    for every registered symbolic input whose condition (every conjunct of
    _create_condition) is among the query's conjuncts."""
    from .keccak_manager import PART, keccak_function_manager as km
    from .solver import _conjuncts
    facts: Dict[Node, tuple] = {}
    for n, xs in km.symbolic_inputs.items():
        if n not in km.interval_hook_for_size:
            continue
        lo = km.interval_hook_for_size[n] * PART
        hashes = frozenset(h.value for c, h in km.concrete_hashes.items() if c.size() == n)
        func, _ = km.get_function(n)
        for x in xs:
            app = func(x).raw
            if app in facts:
                continue
            cond = km._create_condition(x).raw
            if all(c in conj for c in _conjuncts(cond)):
                facts[app] = (lo, lo + PART, hashes)
    return facts


def _differs(key: Node, fact: tuple) -> bool:
    """key (a constant) cannot equal an application with this fact."""
    lo, hi, hashes = fact
    k = key.param
    return (k < lo or k >= hi or k % 64 != 0) and k not in hashes


_OPAQUE = frozenset({"uf", "select", "store", "K", "array"})     # not folded on constants


def _unit(c: Node) -> Optional[tuple]:
    """(var, value) when the conjunct states var == value: eq(var, const), or
    that under the ite(P, 1, 0) wrappers the EVM's ISZERO/EQ words put round it
    (distinct(ite(P,1,0),0), eq(ite(P,1,0),1))."""
    while c.op in ("eq", "distinct") and c.args[0].op == "ite" and c.args[1].op == "const":
        ite, k = c.args
        if ite.args[1].op != "const" or ite.args[2].op != "const" or ite.args[1].param == ite.args[2].param:
            return None
        # P holds exactly when eq(ite, then-value) or distinct(ite, else-value);
        # any other constant leaves P open (distinct(ite(P,1,0), 2) is a tautology)
        holds = k.param == (ite.args[1].param if c.op == "eq" else ite.args[2].param)
        if not holds:
            return None
        c = ite.args[0]
    if c.op == "eq":
        a, b = c.args
        if a.op == "var" and b.op == "const":
            return a, b
        if b.op == "var" and a.op == "const":
            return b, a
    return None


def refutes(conjuncts: Iterable[Node]) -> bool:
    """True when the conjunction is unsatisfiable by the keccak-axiom select
    rewrite above, or by substituting the query's unit equalities (var ==
    const conjuncts: a call value pinned to 0 by the non-payable check against
    a path that needs it positive)."""
    conj = [c for c in conjuncts if c.op != "const"]
    cset = set(conj)
    facts = _keccak_facts(cset)
    memo: Dict[int, Node] = {}
    for c in conj:
        u = _unit(c)
        if u is not None:
            prev = memo.get(id(u[0]))
            if prev is not None and prev is not u[1]:
                return True                    # var == a and var == b, a != b
            memo[id(u[0])] = u[1]
    if not facts and not memo:
        return False

    def select(arr: Node, idx: Node, width: int) -> Optional[Node]:
        fact = facts.get(idx)
        a = arr
        while fact is not None and a.op == "store" and a.args[1].op == "const" and _differs(a.args[1], fact):
            a = a.args[0]
        if a.op == "K":
            return a.args[0]
        return None if a is arr else Node("select", width, (a, idx))

    def rw(n: Node) -> Node:
        r = memo.get(id(n))
        if r is not None:
            return r
        if not n.args:
            return n
        args = tuple(rw(a) for a in n.args)
        if n.op == "select":
            s = select(args[0], args[1], n.width)
            if s is not None:
                memo[id(n)] = s
                return s
        if n.op == "ite" and args[0].op == "const":
            r = args[1] if args[0].param else args[2]
        elif all(a is b for a, b in zip(args, n.args)):
            r = n
        elif n.op in _OPAQUE:
            r = Node(n.op, n.width, args, n.param)
        else:
            r = _fold(n.op, n.width, args, n.param)
        memo[id(n)] = r
        return r

    return any(rw(c) is FALSE for c in conj)
