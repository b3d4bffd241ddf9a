"""CPU ORACLE for KvStore publication decode.

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, as the checker; nothing in openr_amd/ imports it.

A pure-Python restatement of the thrift compact protocol (the wire format of
fbthrift's CompactSerializer, which Decision uses through
readThriftObjStr<...>(value, serializer_) at Decision.cpp:725-726, 745-746)
for the structs the route path consumes:

  PerfEvent / PerfEvents           openr/if/Types.thrift:80-95
  Adjacency                        openr/if/Types.thrift:145-215
  AdjacencyDatabase                openr/if/Types.thrift:223-270
  PrefixMetrics / PrefixEntry      openr/if/Types.thrift:283-408
  PrefixDatabase                   openr/if/Types.thrift:415-430
  BinaryAddress / IpPrefix         openr/if/Network.thrift:49-58

and of the per-key ingestion rules of Decision::updateKeyInLsdb /
deleteKeyFromLsdb (Decision.cpp:710-820), PrefixKey::fromStr
(LsdbTypes.cpp:28-48, LsdbTypes.h:450-458) and getNodeNameFromKey
(LsdbUtil.cpp:691-698).

Parity status: the wire format is pinned by the compact-protocol
specification only. fbthrift (and Apache thrift's Python package) are absent
from this image and the reference holds no serialized AdjacencyDatabase /
PrefixDatabase fixtures, so no reference-produced bytes exist to pin against:
"parity unpinned" for the byte layout. Decoded structs feed
the refcpu oracle's LinkState / PrefixState, which are pinned by the KATs.

Dict shapes follow tests/lsdb.py: addresses are text (socket.inet_ntop, the
form folly::IPAddress::str() prints), prefixes the masked "addr/len" network
string of toIPNetwork(prefix, applyMask=true) (NetworkUtil.h:196-208).
"""

import socket
import struct

CT_STOP, CT_TRUE, CT_FALSE, CT_BYTE, CT_I16, CT_I32, CT_I64 = 0, 1, 2, 3, 4, 5, 6
CT_DOUBLE, CT_BINARY, CT_LIST, CT_SET, CT_MAP, CT_STRUCT, CT_FLOAT = 7, 8, 9, 10, 11, 12, 13

# schema rows: (field id, name, kind, arg, default). kind: bool i16 i32 i64
# str addr prefix metrics struct list-of-struct strlist strset perf.
ADJACENCY = [
    (1, "otherNodeName", "str", None, ""),
    (2, "ifName", "str", None, ""),
    (3, "nextHopV6", "addr", None, ""),
    (4, "metric", "i32", None, 0),
    (5, "nextHopV4", "addr", None, ""),
    (6, "adjLabel", "i32", None, 0),
    (7, "isOverloaded", "bool", None, False),
    (8, "rtt", "i32", None, 0),
    (9, "timestamp", "i64", None, 0),
    (10, "weight", "i64", None, 1),
    (11, "otherIfName", "str", None, ""),
    (12, "adjOnlyUsedByOtherNode", "bool", None, False),
]
ADJ_DB = [
    (1, "thisNodeName", "str", None, ""),
    (2, "isOverloaded", "bool", None, False),
    (3, "adjacencies", "structlist", ADJACENCY, None),
    (4, "nodeLabel", "i32", None, 0),
    (5, "perfEvents", "perf", None, None),  # optional
    (6, "area", "str", None, ""),
    (7, "nodeMetricIncrementVal", "i32", None, 0),
]
METRICS = [
    (1, "version", "i32", None, 1),
    (2, "path_preference", "i32", None, 0),
    (3, "source_preference", "i32", None, 0),
    (4, "distance", "i32", None, 0),
    (5, "drain_metric", "i32", None, 0),
]
PREFIX_ENTRY = [
    (1, "prefix", "prefix", None, None),
    (2, "type", "i32", None, 0),
    (4, "forwardingType", "i32", None, 0),
    (7, "forwardingAlgorithm", "i32", None, 0),
    (8, "minNexthop", "i64", None, None),  # optional
    (10, "metrics", "struct", METRICS, None),
    (11, "tags", "strset", None, None),
    (12, "area_stack", "strlist", None, None),
    (13, "weight", "i64", None, None),  # optional
]
PREFIX_DB = [
    (1, "thisNodeName", "str", None, ""),
    (3, "prefixEntries", "structlist", PREFIX_ENTRY, None),
    (4, "perfEvents", "perf", None, None),  # optional
    (5, "deletePrefix", "bool", None, False),
]
PERF_EVENT = [
    (1, "nodeName", "str", None, ""),
    (2, "eventDescr", "str", None, ""),
    (3, "unixTs", "i64", None, 0),
]

WIRE = {"bool": (CT_TRUE, CT_FALSE), "i16": (CT_I16,), "i32": (CT_I32,), "i64": (CT_I64,),
        "str": (CT_BINARY,), "addr": (CT_STRUCT,), "prefix": (CT_STRUCT,),
        "struct": (CT_STRUCT,), "structlist": (CT_LIST,), "strlist": (CT_LIST,),
        "strset": (CT_SET,), "perf": (CT_STRUCT,)}


class DecodeError(ValueError):
    pass


# ----------------------------------------------------------------- addresses --
def addr_to_text(raw):
    if len(raw) == 0:
        return ""
    if len(raw) == 4:
        return socket.inet_ntop(socket.AF_INET, raw)
    if len(raw) == 16:
        return socket.inet_ntop(socket.AF_INET6, raw)
    raise DecodeError("BinaryAddress.addr must be 4 or 16 bytes")


def text_to_addr(text):
    if not text:
        return b""
    fam = socket.AF_INET6 if ":" in text else socket.AF_INET
    return socket.inet_pton(fam, text)


def prefix_string(raw, plen):
    """IpPrefix as advertised (host bits kept): what Decision keeps in the
    stored entry (Decision.cpp:758-778). Rejects what toIPNetwork rejects."""
    if len(raw) not in (4, 16):
        raise DecodeError("prefix address must be 4 or 16 bytes")
    if plen < 0 or plen > 8 * len(raw):
        raise DecodeError("prefix length out of range")
    return "%s/%d" % (addr_to_text(raw), plen)


def network_of_text(text):
    """toIPNetwork(entry.prefix) of an "addr/len" text: the PrefixState key."""
    addr, _, plen = text.rpartition("/")
    return network_string(text_to_addr(addr), int(plen))


def network_string(raw, plen):
    """toIPNetwork(IpPrefix, applyMask=true) printed as addr/len."""
    if len(raw) not in (4, 16):
        raise DecodeError("prefix address must be 4 or 16 bytes")
    bits = 8 * len(raw)
    if plen < 0 or plen > bits:
        raise DecodeError("prefix length out of range")
    v = int.from_bytes(raw, "big")
    mask = ((1 << bits) - 1) ^ ((1 << (bits - plen)) - 1)
    return "%s/%d" % (addr_to_text((v & mask).to_bytes(len(raw), "big")), plen)


# ------------------------------------------------------------------ decoding --
class _Reader:
    def __init__(self, b):
        self.b = bytes(b)
        self.i = 0

    def byte(self):
        if self.i >= len(self.b):
            raise DecodeError("truncated input")
        v = self.b[self.i]
        self.i += 1
        return v

    def varint(self):
        v = shift = 0
        while True:
            c = self.byte()
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7
            if shift >= 70:
                raise DecodeError("varint too long")

    def zz(self, bits):
        u = self.varint()
        v = (u >> 1) ^ -(u & 1)
        if not -(1 << (bits - 1)) <= v < (1 << (bits - 1)):
            raise DecodeError("integer out of range")
        return v

    def bytes_(self):
        n = self.varint()
        if n > len(self.b) - self.i:
            raise DecodeError("string past end of input")
        s = self.b[self.i:self.i + n]
        self.i += n
        return s

    def list_header(self):
        h = self.byte()
        n = h >> 4
        if n == 15:
            n = self.varint()
        if n > len(self.b) - self.i:
            raise DecodeError("container size past end of input")
        return h & 0x0F, n

    def fields(self):
        last = 0
        while True:
            h = self.byte()
            if h == CT_STOP:
                return
            t, d = h & 0x0F, h >> 4
            fid = last + d if d else self.zz(16)
            last = fid
            yield fid, t

    def skip(self, t, depth=0):
        if depth > 64:
            raise DecodeError("nesting too deep")
        if t in (CT_TRUE, CT_FALSE):
            return
        if t == CT_BYTE:
            self.i += 1
        elif t in (CT_I16, CT_I32, CT_I64):
            self.varint()
        elif t == CT_DOUBLE:
            self.i += 8
        elif t == CT_FLOAT:
            self.i += 4
        elif t == CT_BINARY:
            self.bytes_()
        elif t in (CT_LIST, CT_SET):
            et, n = self.list_header()
            for _ in range(n):
                self.skip_elem(et, depth + 1)
        elif t == CT_MAP:
            n = self.varint()
            if n:
                kv = self.byte()
                for _ in range(n):
                    self.skip_elem(kv >> 4, depth + 1)
                    self.skip_elem(kv & 0x0F, depth + 1)
        elif t == CT_STRUCT:
            for _, ft in self.fields():
                self.skip(ft, depth + 1)
        else:
            raise DecodeError("unknown wire type %d" % t)
        if self.i > len(self.b):
            raise DecodeError("truncated input")

    def skip_elem(self, t, depth):
        if t in (CT_TRUE, CT_FALSE):
            if self.byte() not in (0, 1, 2):
                raise DecodeError("bad bool element")
            return
        self.skip(t, depth)


def _read_struct(r, schema):
    out = {name: (dict(d) if isinstance(d, dict) else d) for _, name, _, _, d in schema}
    rows = {fid: (name, kind, arg) for fid, name, kind, arg, _ in schema}
    for name, kind, arg in ((n, k, a) for _, n, k, a, _ in schema):
        if kind == "struct":
            out[name] = _read_struct(_Reader(b"\x00"), arg)  # defaults
        elif kind in ("structlist", "strlist", "strset"):
            out[name] = []
    for fid, t in r.fields():
        row = rows.get(fid)
        if row is None or t not in WIRE[row[1]]:
            r.skip(t, 1)
            continue
        name, kind, arg = row
        if kind == "bool":
            out[name] = t == CT_TRUE
        elif kind == "i16":
            out[name] = r.zz(16)
        elif kind == "i32":
            out[name] = r.zz(32)
        elif kind == "i64":
            out[name] = r.zz(64)
        elif kind == "str":
            out[name] = r.bytes_().decode("utf-8", "surrogateescape")
        elif kind == "addr":
            out[name] = addr_to_text(_read_binary_address(r))
        elif kind == "prefix":
            addr, plen = b"", 0
            for f2, t2 in r.fields():
                if f2 == 1 and t2 == CT_STRUCT:
                    addr = _read_binary_address(r)
                elif f2 == 2 and t2 == CT_I16:
                    plen = r.zz(16)
                else:
                    r.skip(t2, 2)
            out[name] = prefix_string(addr, plen)
        elif kind == "struct":
            out[name] = _read_struct(r, arg)
        elif kind in ("structlist", "strlist", "strset"):
            et, n = r.list_header()
            want = CT_STRUCT if kind == "structlist" else CT_BINARY
            vals = []
            for _ in range(n):
                if et != want:
                    r.skip_elem(et, 2)
                elif kind == "structlist":
                    vals.append(_read_struct(r, arg))
                else:
                    vals.append(r.bytes_().decode("utf-8", "surrogateescape"))
            out[name] = sorted(set(vals)) if kind == "strset" else vals
        elif kind == "perf":
            evs = []
            for f2, t2 in r.fields():
                if f2 == 1 and t2 == CT_LIST:
                    et, n = r.list_header()
                    for _ in range(n):
                        if et != CT_STRUCT:
                            r.skip_elem(et, 2)
                            continue
                        ev = _read_struct(r, PERF_EVENT)
                        evs.append((ev["nodeName"], ev["eventDescr"], ev["unixTs"]))
                else:
                    r.skip(t2, 2)
            out[name] = evs
    return out


def _read_binary_address(r):
    addr = b""
    for fid, t in r.fields():
        if fid == 1 and t == CT_BINARY:
            addr = r.bytes_()
        else:
            r.skip(t, 2)
    return addr


def decode_adj_db(b):
    return _read_struct(_Reader(b), ADJ_DB)


def decode_prefix_db(b):
    return _read_struct(_Reader(b), PREFIX_DB)


# ------------------------------------------------------------------ encoding --
def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _zz(v):
    return _varint(((v << 1) ^ (v >> 63)) & ((1 << 64) - 1))


def _bin(s):
    if isinstance(s, str):
        s = s.encode("utf-8", "surrogateescape")
    return _varint(len(s)) + s


def _hdr(last, fid, t):
    d = fid - last
    return bytes([(d << 4) | t]) if 0 < d <= 15 else bytes([t]) + _zz(fid)


def _list_hdr(et, n):
    return bytes([(n << 4) | et]) if n < 15 else bytes([0xF0 | et]) + _varint(n)


def _write_struct(d, schema, order=None):
    rows = sorted(schema) if order is None else [r for k in order for r in schema if r[0] == k]
    out, last = bytearray(), 0
    for fid, name, kind, arg, dflt in rows:
        v = d.get(name, dflt)
        if v is None and kind in ("i64", "perf", "prefix"):
            continue  # optional and unset
        if kind == "bool":
            out += _hdr(last, fid, CT_TRUE if v else CT_FALSE)
        elif kind in ("i16", "i32", "i64"):
            out += _hdr(last, fid, WIRE[kind][0]) + _zz(v)
        elif kind == "str":
            out += _hdr(last, fid, CT_BINARY) + _bin(v or "")
        elif kind == "addr":
            out += _hdr(last, fid, CT_STRUCT) + _hdr(0, 1, CT_BINARY) + _bin(text_to_addr(v)) + b"\x00"
        elif kind == "prefix":
            a, plen = v.rsplit("/", 1)
            out += _hdr(last, fid, CT_STRUCT)
            out += _hdr(0, 1, CT_STRUCT) + _hdr(0, 1, CT_BINARY) + _bin(text_to_addr(a)) + b"\x00"
            out += _hdr(1, 2, CT_I16) + _zz(int(plen)) + b"\x00"
        elif kind == "struct":
            out += _hdr(last, fid, CT_STRUCT) + _write_struct(v or {}, arg)
        elif kind == "structlist":
            v = v or []
            out += _hdr(last, fid, CT_LIST) + _list_hdr(CT_STRUCT, len(v))
            for x in v:
                out += _write_struct(x, arg)
        elif kind in ("strlist", "strset"):
            v = list(v or [])
            if kind == "strset":
                v = sorted(set(v), key=lambda s: s.encode("utf-8", "surrogateescape"))
            out += _hdr(last, fid, CT_LIST if kind == "strlist" else CT_SET)
            out += _list_hdr(CT_BINARY, len(v))
            for s in v:
                out += _bin(s)
        elif kind == "perf":
            out += _hdr(last, fid, CT_STRUCT) + _hdr(0, 1, CT_LIST) + _list_hdr(CT_STRUCT, len(v))
            for n, e, ts in v:
                out += _write_struct(dict(nodeName=n, eventDescr=e, unixTs=ts), PERF_EVENT)
            out += b"\x00"
        last = fid
    out.append(CT_STOP)
    return bytes(out)


def encode_adj_db(d, order=None):
    d = dict(d)
    d.setdefault("perfEvents", None)
    return _write_struct(d, ADJ_DB, order)


def encode_prefix_db(d, order=None):
    return _write_struct(d, PREFIX_DB, order)


# ------------------------------------------------------- Decision key rules --
def get_node_name_from_key(key):
    """LsdbUtil.cpp:691-698 (folly::split on ':' then element 1)."""
    parts = key.split(":")
    return parts[1] if len(parts) >= 2 else ""


def parse_prefix_key(key):
    """PrefixKey::fromStr (LsdbTypes.cpp:28-48) -> (node, network) or None."""
    import re
    m = re.fullmatch(r"prefix:([a-zA-Z\d.\-_]+):\[([a-fA-F\d.:]+)/(\d{1,3})\]", key)
    if not m:
        return None
    node, ip, plen = m.group(1), m.group(2), int(m.group(3))
    try:
        return node, network_string(text_to_addr(ip), plen)
    except (OSError, DecodeError):
        return None


def update_key_in_lsdb(my_node, areas, area, link_state, prefix_state, key, value,
                       in_initialization=False):
    """Decision::updateKeyInLsdb (Decision.cpp:710-785) over refcpu objects.
    Returns (kind, nodeName, payload) with kind as in lsdb_codec.h."""
    if value is None:
        return 0, "", None
    try:
        if key.startswith("adj:"):
            db = decode_adj_db(value)
            db["area"] = area
            db.pop("perfEvents", None)
            return 1, db["thisNodeName"], link_state.updateAdjacencyDatabase(db, area, in_initialization)
        if key.startswith("prefix:"):
            db = decode_prefix_db(value)
            if len(db["prefixEntries"]) != 1:
                return 3, db["thisNodeName"], None
            e = db["prefixEntries"][0]
            if db["thisNodeName"] == my_node and e["area_stack"] and e["area_stack"][-1] in areas:
                return 0, "", None
            node = db["thisNodeName"]
            if not e["prefix"]:  # default IpPrefix: toIPNetwork throws
                return 3, "", None
            if db["deletePrefix"]:  # PrefixKey(node, toIPNetwork(prefix), area)
                return 2, node, set(prefix_state.deletePrefix(node, area, network_of_text(e["prefix"])))
            return 2, node, set(prefix_state.updatePrefix(node, area, e))
    except DecodeError:
        return 3, "", None
    return 0, "", None


def delete_key_from_lsdb(area, link_state, prefix_state, key):
    """Decision::deleteKeyFromLsdb (Decision.cpp:787-818)."""
    if key.startswith("adj:"):
        node = get_node_name_from_key(key)
        return 1, node, link_state.deleteAdjacencyDatabase(node)
    if key.startswith("prefix:"):
        pk = parse_prefix_key(key)
        if pk is None:
            return 3, "", None
        return 2, pk[0], set(prefix_state.deletePrefix(pk[0], area, pk[1]))
    return 0, "", None


class PendingUpdates:
    """DecisionPendingUpdates (Decision.h:40-105, Decision.cpp:35-60) without
    perf events."""

    def __init__(self, my_node):
        self.me, self.count, self.full, self.prefixes = my_node, 0, False, set()

    def apply(self, kind, node, payload):
        if kind == 1:
            self.full |= bool(payload["topologyChanged"] or payload["nodeLabelChanged"]
                              or (payload["linkAttributesChanged"] and node == self.me))
            self.count += 1
        elif kind == 2:
            self.prefixes |= set(payload)
            self.count += 1


def process_publication(my_node, area_link_states, make_link_state, prefix_state, area,
                        key_vals, expired_keys, pending, in_initialization=False):
    """Decision::processPublication (Decision.cpp:821-846); area_link_states
    is a plain dict area -> LinkState, key_vals (key, bytes|None) pairs
    applied as a std::map (sorted keys, last duplicate wins)."""
    if area not in area_link_states:
        area_link_states[area] = make_link_state(area, my_node)
    ls = area_link_states[area]
    if not key_vals and not expired_keys:
        return
    areas = set(area_link_states)
    for key, val in sorted(dict(key_vals).items()):
        pending.apply(*update_key_in_lsdb(my_node, areas, area, ls, prefix_state, key, val,
                                          in_initialization))
    for key in expired_keys:
        pending.apply(*delete_key_from_lsdb(area, ls, prefix_state, key))
