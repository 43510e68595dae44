"""Control-plane message vocabulary and wire framing.

Same logical message set as the reference (utils.py:11-23 ``Type`` plus the
METADATA push), but structured: every message is a msgpack map
``{"t": <type>, "src": <node>, ...fields}`` sent as a length-prefixed frame
(4-byte big-endian length).  This fixes the reference's ``<SEPARATOR>``-joined
strings read with a single ``recv(4096)`` (truncation of RESULT / METADATA,
SURVEY.md A4).
"""
from __future__ import annotations

import struct

import msgpack


class Type:
    PING = "Ping"
    PONG = "Pong"
    JOIN = "Join"
    LEAVE = "Leave"
    PUT = "PUT"
    GET = "GET"
    DELETE = "DELETE"
    LS = "LS"
    STORE = "STORE"
    GET_VERSIONS = "GET-VERSIONS"
    REPLICATE = "REPLICATE"          # master -> replica: store (name, version, bytes)
    UNLINK = "UNLINK"                # master -> replica: remove all versions
    FETCH = "FETCH"                  # master -> replica: read (name, version)
    HBM_HAS = "HBM_HAS"              # node -> SDFS master: I hold / dropped this file in HBM
    FETCH_HBM = "FETCH_HBM"          # node -> node: IPC handle of your HBM copy (GPU-to-GPU copy)
    INFERENCE = "INFERENCE"          # client -> coordinator: a query
    JOB = "JOB"                      # coordinator -> worker: one chunk
    RESULT = "RESULT"                # worker -> coordinator (+ standby): top-1 of a chunk
    METADATA = "METADATA"            # coordinator -> standby: job-state snapshot / delta
    PROMOTE = "PROMOTE"              # standby -> all: I am the coordinator now (new epoch)
    STATS = "STATS"                  # shell views (c1/c2/c4/cq/cvm) from the coordinator
    GREP = "GREP"                    # distributed log grep (MP1 replacement)
    REPLY = "REPLY"                  # response to a request (carries "rid")
    KILL = "KILL"                    # fault injection
    GROUP_FORM = "GROUP_FORM"        # coordinator -> members: join collective-group epoch N
    ROUND = "ROUND"                  # coordinator -> member: its descriptor row of round k (or STOP)
    RESULTS = "RESULTS"              # coordinator -> standby: every chunk of one finished round


Status_RUNNING = "RUNNING"
Status_LEAVE = "LEAVE"

_HDR = struct.Struct(">I")
MAX_FRAME = 1 << 31


def encode(msg: dict) -> bytes:
    body = msgpack.packb(msg, use_bin_type=True)
    if len(body) >= MAX_FRAME:
        raise ValueError("frame too large")
    return _HDR.pack(len(body)) + body


def decode(body: bytes) -> dict:
    return msgpack.unpackb(body, raw=False, strict_map_key=False)


class FrameReader:
    """Incremental decoder for a byte stream of length-prefixed frames."""

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes) -> list[dict]:
        self.buf += data
        out = []
        while len(self.buf) >= 4:
            (n,) = _HDR.unpack_from(self.buf, 0)
            if len(self.buf) < 4 + n:
                break
            out.append(decode(bytes(self.buf[4:4 + n])))
            del self.buf[:4 + n]
        return out
