"""Host-ring placement helpers (reference utils.py:30-61).

The reference hard-codes a 10-host ring ``fa22-cs425-01{01..10}``.  Here the
ring is the sorted list of node names of the cluster (one per GPU); the
helpers keep the reference semantics over that list:

  replica_neighbors(n)  the successors of n with wrap-around, ending at n itself
                        (reference: host 5 -> 6,7,8,9,10,1,2,3,4,5)
  neighbors(n)          every node except n
  file_neighbors(k, r)  r consecutive ring nodes starting at index k
                        (reference: k..k+4 -> 4-5 replicas; here exactly r)
"""
from __future__ import annotations


def replica_neighbors(node: str, ring: list[str]) -> list[str]:
    ring = sorted(ring)
    if node not in ring:
        ring = sorted(ring + [node])
    i = ring.index(node)
    return ring[i + 1:] + ring[:i + 1]


def neighbors(node: str, ring: list[str]) -> list[str]:
    return [n for n in sorted(ring) if n != node]


def file_neighbors(k: int, ring: list[str], r: int) -> list[str]:
    ring = sorted(ring)
    if not ring:
        return []
    r = min(r, len(ring))
    return [ring[(k + i) % len(ring)] for i in range(r)]
