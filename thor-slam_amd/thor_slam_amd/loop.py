"""Host-side rules of the asynchronous loop closure shared by ``HipSlamEngine`` (spec:
``oracle/numpy_loop.py`` ``LoopPolicy``, which restates them independently)."""

from __future__ import annotations


def span_edges(edges: list, a: int, b: int) -> list[int]:
    """Indices of the pose-graph edges (x, y), x < y, with both ends in the node span [a, b], in
    the canonical order (y, x): the span solve's summation order does not depend on when a loop
    edge was recorded (oracle ``numpy_loop.span_edges``)."""
    return sorted((e for e, (x, y) in enumerate(edges) if a <= x and y <= b), key=lambda e: (edges[e][1], edges[e][0]))
