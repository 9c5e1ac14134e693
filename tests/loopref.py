"""Pure-Python restatement of BoundedLoopsStrategy.get_loop_count
(laser/ethereum/strategy/extensions/bounded_loops.py:49-113) — test oracle for
the C oracle and the device.  Python ints, so the OR-of-shifted-addresses hash is
computed exactly as the reference computes it."""


def segment_hash(trace, i, j):
    key = 0
    for itr in range(i, j):
        key |= trace[itr] << ((itr - i) * 8)
    return key


def loop_count(trace):
    n = len(trace)
    start = None
    for i in range(n - 3, 0, -1):
        if trace[i] == trace[-2] and trace[i + 1] == trace[-1]:
            start = i
            break
    if start is None:
        return 0
    key = segment_hash(trace, start + 1, n - 1)
    size = n - start - 2
    count, j = 1, start + 1
    while j >= 0:
        if segment_hash(trace, j, j + size) != key:
            break
        count += 1
        j -= size
    return count
