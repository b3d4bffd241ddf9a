// lsdb_codec.cpp — compact-protocol decode of KvStore publications and the
// Decision per-key ingestion step (§8(f) f4). See lsdb_codec.h for the
// reference interfaces replaced.
//
// Wire format (thrift compact protocol, as written by fbthrift's
// CompactSerializer): a struct is a run of field headers closed by a 0 byte.
// A header byte carries (id delta << 4 | type) when 1 <= delta <= 15, else
// (type) followed by the zigzag-varint i16 id. Booleans live in the header's
// type nibble (1 true / 2 false). i16/i32/i64 are zigzag varints, strings and
// binaries a varint length + bytes, lists/sets a (size << 4 | elem) byte
// (size >= 15: 0xF0 | elem then a varint size), maps a varint size then
// (key << 4 | value) when non-empty.
#include "lsdb_codec.h"

#include <algorithm>
#include <chrono>

#include <arpa/inet.h>

#include <cstring>

namespace openr_amd {
namespace {

enum CType : uint8_t {
  CT_STOP = 0,
  CT_TRUE = 1,
  CT_FALSE = 2,
  CT_BYTE = 3,
  CT_I16 = 4,
  CT_I32 = 5,
  CT_I64 = 6,
  CT_DOUBLE = 7,
  CT_BINARY = 8,
  CT_LIST = 9,
  CT_SET = 10,
  CT_MAP = 11,
  CT_STRUCT = 12,
  CT_FLOAT = 13,
};

constexpr int kMaxDepth = 64;

[[noreturn]] void fail(const char* what) { throw LsdbDecodeError(what); }

class Reader {
 public:
  explicit Reader(std::string_view b)
      : p_(reinterpret_cast<const uint8_t*>(b.data())), e_(p_ + b.size()) {}

  uint8_t byte() {
    if (p_ >= e_) fail("compact: truncated input");
    return *p_++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 70; shift += 7) {
      uint8_t b = byte();
      v |= uint64_t(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    fail("compact: varint too long");
  }
  int64_t zz64() {
    uint64_t u = varint();
    return int64_t(u >> 1) ^ -int64_t(u & 1);
  }
  int32_t zz32() {
    int64_t v = zz64();
    if (v < INT32_MIN || v > INT32_MAX) fail("compact: i32 out of range");
    return int32_t(v);
  }
  int16_t zz16() {
    int64_t v = zz64();
    if (v < INT16_MIN || v > INT16_MAX) fail("compact: i16 out of range");
    return int16_t(v);
  }
  std::string_view bytes() {
    uint64_t n = varint();
    if (n > uint64_t(e_ - p_)) fail("compact: string past end of input");
    std::string_view s(reinterpret_cast<const char*>(p_), size_t(n));
    p_ += n;
    return s;
  }
  void skipN(uint64_t n) {
    if (n > uint64_t(e_ - p_)) fail("compact: truncated input");
    p_ += n;
  }
  // list / set header -> (elem type, size)
  std::pair<uint8_t, uint32_t> listHeader() {
    uint8_t h = byte();
    uint64_t n = h >> 4;
    if (n == 15) n = varint();
    // every element occupies at least one byte on the wire
    if (n > uint64_t(e_ - p_)) fail("compact: container size past end of input");
    return {uint8_t(h & 0x0f), uint32_t(n)};
  }

  // field header; returns false at the struct's stop byte
  bool field(int16_t& lastId, int16_t& id, uint8_t& type) {
    uint8_t h = byte();
    if (h == CT_STOP) return false;
    type = h & 0x0f;
    uint8_t delta = h >> 4;
    id = delta ? int16_t(lastId + delta) : zz16();
    lastId = id;
    return true;
  }

  bool boolElem() {
    uint8_t b = byte();
    // fbthrift writes 1 / 2 (CT_TRUE / CT_FALSE); accept 0 as false too
    if (b == CT_TRUE) return true;
    if (b == CT_FALSE || b == 0) return false;
    fail("compact: bad bool element");
  }

  void skip(uint8_t type, int depth = 0) {
    if (depth > kMaxDepth) fail("compact: nesting too deep");
    switch (type) {
      case CT_TRUE:
      case CT_FALSE:
        return;  // field-header bool: value is in the type nibble
      case CT_BYTE:
        skipN(1);
        return;
      case CT_I16:
      case CT_I32:
      case CT_I64:
        varint();
        return;
      case CT_DOUBLE:
        skipN(8);
        return;
      case CT_FLOAT:
        skipN(4);
        return;
      case CT_BINARY:
        bytes();
        return;
      case CT_LIST:
      case CT_SET: {
        auto [et, n] = listHeader();
        for (uint32_t i = 0; i < n; ++i) skipElem(et, depth + 1);
        return;
      }
      case CT_MAP: {
        uint64_t n = varint();
        if (n == 0) return;
        if (n > uint64_t(e_ - p_)) fail("compact: map size past end of input");
        uint8_t kv = byte();
        for (uint64_t i = 0; i < n; ++i) {
          skipElem(kv >> 4, depth + 1);
          skipElem(kv & 0x0f, depth + 1);
        }
        return;
      }
      case CT_STRUCT: {
        int16_t last = 0, id;
        uint8_t t;
        while (field(last, id, t)) skip(t, depth + 1);
        return;
      }
      default:
        fail("compact: unknown wire type");
    }
  }
  // container elements: bools take a byte of their own
  void skipElem(uint8_t type, int depth) {
    if (type == CT_TRUE || type == CT_FALSE) {
      boolElem();
      return;
    }
    skip(type, depth);
  }

  bool done() const { return p_ == e_; }

 private:
  const uint8_t* p_;
  const uint8_t* e_;
};

bool isBoolType(uint8_t t) { return t == CT_TRUE || t == CT_FALSE; }

// BinaryAddress (Network.thrift:49-52) -> raw addr bytes (ifName dropped)
std::string_view readBinaryAddress(Reader& r) {
  std::string_view addr;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 1 && t == CT_BINARY) {
      addr = r.bytes();
    } else {
      r.skip(t, 1);
    }
  }
  return addr;
}

std::string readAddressText(Reader& r) {
  return binaryAddressToString(readBinaryAddress(r));
}

void readPerfEvents(Reader& r, std::vector<PerfEvent>& out) {  // Types.thrift:80-95
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 1 && t == CT_LIST) {
      auto [et, n] = r.listHeader();
      if (et != CT_STRUCT) {
        for (uint32_t i = 0; i < n; ++i) r.skipElem(et, 2);
        continue;
      }
      out.reserve(n);
      for (uint32_t i = 0; i < n; ++i) {
        PerfEvent ev;
        int16_t l2 = 0, id2;
        uint8_t t2;
        while (r.field(l2, id2, t2)) {
          if (id2 == 1 && t2 == CT_BINARY) ev.nodeName = r.bytes();
          else if (id2 == 2 && t2 == CT_BINARY) ev.eventDescr = r.bytes();
          else if (id2 == 3 && t2 == CT_I64) ev.unixTs = r.zz64();
          else r.skip(t2, 3);
        }
        out.push_back(std::move(ev));
      }
    } else {
      r.skip(t, 1);
    }
  }
}

Adjacency readAdjacency(Reader& r) {  // Types.thrift:145-215
  Adjacency a;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1:
        if (t == CT_BINARY) { a.otherNodeName = r.bytes(); continue; }
        break;
      case 2:
        if (t == CT_BINARY) { a.ifName = r.bytes(); continue; }
        break;
      case 3:
        if (t == CT_STRUCT) { a.nextHopV6 = readAddressText(r); continue; }
        break;
      case 5:
        if (t == CT_STRUCT) { a.nextHopV4 = readAddressText(r); continue; }
        break;
      case 4:
        if (t == CT_I32) { a.metric = r.zz32(); continue; }
        break;
      case 6:
        if (t == CT_I32) { a.adjLabel = r.zz32(); continue; }
        break;
      case 7:
        if (isBoolType(t)) { a.isOverloaded = t == CT_TRUE; continue; }
        break;
      case 8:
        if (t == CT_I32) { a.rtt = r.zz32(); continue; }
        break;
      case 9:
        if (t == CT_I64) { a.timestamp = r.zz64(); continue; }
        break;
      case 10:
        if (t == CT_I64) { a.weight = r.zz64(); continue; }
        break;
      case 11:
        if (t == CT_BINARY) { a.otherIfName = r.bytes(); continue; }
        break;
      case 12:
        if (isBoolType(t)) { a.adjOnlyUsedByOtherNode = t == CT_TRUE; continue; }
        break;
    }
    r.skip(t, 1);
  }
  return a;
}

// The entry keeps the IpPrefix as advertised (host bits included), the way
// Decision stores the raw thrift entry (Decision.cpp:758-778); `network`,
// when asked for, receives toIPNetwork(prefix) (applyMask = true), the
// PrefixState key. An address toIPNetwork rejects (not 4 / 16 bytes, length
// out of range) throws here, so the key is dropped as Decision.cpp:781-784
// drops it.
std::string readIpPrefix(Reader& r, std::string* network) {  // Network.thrift:55-58
  std::string addr;
  int16_t len = 0;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 1 && t == CT_STRUCT) addr = std::string(readBinaryAddress(r));
    else if (id == 2 && t == CT_I16) len = r.zz16();
    else r.skip(t, 2);
  }
  std::string text = ipPrefixToString(addr, len);  // validates size and length
  if (network) {
    // no host bits set (the usual advertisement): the network prints the same
    bool masked = true;
    for (int bit = len; bit < int(addr.size()) * 8 && masked; ++bit) {
      masked = !(uint8_t(addr[size_t(bit >> 3)]) & (0x80u >> (bit & 7)));
    }
    *network = masked ? text : ipPrefixToNetworkString(addr, len);
  }
  return text;
}

void readMetrics(Reader& r, PrefixMetrics& m) {  // Types.thrift:287-317
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (t == CT_I32 && id >= 1 && id <= 5) {
      int32_t v = r.zz32();
      switch (id) {
        case 1: m.version = v; break;
        case 2: m.path_preference = v; break;
        case 3: m.source_preference = v; break;
        case 4: m.distance = v; break;
        case 5: m.drain_metric = v; break;
      }
    } else {
      r.skip(t, 2);
    }
  }
}

void readStringList(Reader& r, uint8_t t, std::vector<std::string>* vec,
                    std::set<std::string>* set) {
  auto [et, n] = r.listHeader();
  if (et != CT_BINARY) {
    for (uint32_t i = 0; i < n; ++i) r.skipElem(et, 2);
    return;
  }
  (void)t;
  for (uint32_t i = 0; i < n; ++i) {
    std::string_view s = r.bytes();
    if (vec) vec->emplace_back(s);
    else set->emplace(s);
  }
}

PrefixEntry readPrefixEntry(Reader& r, std::string* network) {  // Types.thrift:349-408
  PrefixEntry e;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1:
        if (t == CT_STRUCT) { e.prefix = readIpPrefix(r, network); continue; }
        break;
      case 2:
        if (t == CT_I32) { e.type = r.zz32(); continue; }
        break;
      case 4:
        if (t == CT_I32) { e.forwardingType = r.zz32(); continue; }
        break;
      case 7:
        if (t == CT_I32) { e.forwardingAlgorithm = r.zz32(); continue; }
        break;
      case 8:
        if (t == CT_I64) { e.minNexthop = r.zz64(); continue; }
        break;
      case 10:
        if (t == CT_STRUCT) { readMetrics(r, e.metrics); continue; }
        break;
      case 11:
        if (t == CT_SET) { readStringList(r, t, nullptr, &e.tags); continue; }
        break;
      case 12:
        if (t == CT_LIST) { readStringList(r, t, &e.area_stack, nullptr); continue; }
        break;
      case 13:
        if (t == CT_I64) { e.weight = r.zz64(); continue; }
        break;
    }
    r.skip(t, 1);
  }
  return e;
}

// ------------------------------------------------------------- writer --
class Writer {
 public:
  std::string out;
  void byte(uint8_t b) { out.push_back(char(b)); }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      byte(uint8_t(v | 0x80));
      v >>= 7;
    }
    byte(uint8_t(v));
  }
  void zz(int64_t v) { varint((uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
  void bytes(std::string_view s) {
    varint(s.size());
    out.append(s.data(), s.size());
  }
  void field(int16_t& last, int16_t id, uint8_t type) {
    int d = id - last;
    if (d > 0 && d <= 15) {
      byte(uint8_t(d << 4 | type));
    } else {
      byte(type);
      zz(id);
    }
    last = id;
  }
  void boolField(int16_t& last, int16_t id, bool v) { field(last, id, v ? CT_TRUE : CT_FALSE); }
  void listHeader(uint8_t et, size_t n) {
    if (n < 15) {
      byte(uint8_t(n << 4 | et));
    } else {
      byte(uint8_t(0xf0 | et));
      varint(n);
    }
  }
  void stop() { byte(CT_STOP); }
};

void writeBinaryAddress(Writer& w, const std::string& text) {
  int16_t last = 0;
  w.field(last, 1, CT_BINARY);
  w.bytes(stringToBinaryAddress(text));
  w.stop();
}

void writeAdjacency(Writer& w, const Adjacency& a) {
  int16_t l = 0;
  w.field(l, 1, CT_BINARY); w.bytes(a.otherNodeName);
  w.field(l, 2, CT_BINARY); w.bytes(a.ifName);
  w.field(l, 3, CT_STRUCT); writeBinaryAddress(w, a.nextHopV6);
  w.field(l, 4, CT_I32); w.zz(a.metric);
  w.field(l, 5, CT_STRUCT); writeBinaryAddress(w, a.nextHopV4);
  w.field(l, 6, CT_I32); w.zz(a.adjLabel);
  w.boolField(l, 7, a.isOverloaded);
  w.field(l, 8, CT_I32); w.zz(a.rtt);
  w.field(l, 9, CT_I64); w.zz(a.timestamp);
  w.field(l, 10, CT_I64); w.zz(a.weight);
  w.field(l, 11, CT_BINARY); w.bytes(a.otherIfName);
  w.boolField(l, 12, a.adjOnlyUsedByOtherNode);
  w.stop();
}

void writePerfEvents(Writer& w, const std::vector<PerfEvent>& evs) {
  int16_t l = 0;
  w.field(l, 1, CT_LIST);
  w.listHeader(CT_STRUCT, evs.size());
  for (const auto& ev : evs) {
    int16_t l2 = 0;
    w.field(l2, 1, CT_BINARY); w.bytes(ev.nodeName);
    w.field(l2, 2, CT_BINARY); w.bytes(ev.eventDescr);
    w.field(l2, 3, CT_I64); w.zz(ev.unixTs);
    w.stop();
  }
  w.stop();
}

void writePrefixEntry(Writer& w, const PrefixEntry& e) {
  int16_t l = 0;
  auto slash = e.prefix.rfind('/');
  if (slash == std::string::npos) throw std::invalid_argument("prefix without length: " + e.prefix);
  w.field(l, 1, CT_STRUCT);
  {
    int16_t l2 = 0;
    w.field(l2, 1, CT_STRUCT); writeBinaryAddress(w, e.prefix.substr(0, slash));
    w.field(l2, 2, CT_I16); w.zz(std::stoi(e.prefix.substr(slash + 1)));
    w.stop();
  }
  w.field(l, 2, CT_I32); w.zz(e.type);
  w.field(l, 4, CT_I32); w.zz(e.forwardingType);
  w.field(l, 7, CT_I32); w.zz(e.forwardingAlgorithm);
  if (e.minNexthop) { w.field(l, 8, CT_I64); w.zz(*e.minNexthop); }
  w.field(l, 10, CT_STRUCT);
  {
    int16_t l2 = 0;
    w.field(l2, 1, CT_I32); w.zz(e.metrics.version);
    w.field(l2, 2, CT_I32); w.zz(e.metrics.path_preference);
    w.field(l2, 3, CT_I32); w.zz(e.metrics.source_preference);
    w.field(l2, 4, CT_I32); w.zz(e.metrics.distance);
    w.field(l2, 5, CT_I32); w.zz(e.metrics.drain_metric);
    w.stop();
  }
  w.field(l, 11, CT_SET);
  w.listHeader(CT_BINARY, e.tags.size());
  for (const auto& s : e.tags) w.bytes(s);
  w.field(l, 12, CT_LIST);
  w.listHeader(CT_BINARY, e.area_stack.size());
  for (const auto& s : e.area_stack) w.bytes(s);
  if (e.weight) { w.field(l, 13, CT_I64); w.zz(*e.weight); }
  w.stop();
}

bool parseAddress(const std::string& text, unsigned char buf[16], int& family) {
  if (text.find(':') != std::string::npos) {
    family = AF_INET6;
    return inet_pton(AF_INET6, text.c_str(), buf) == 1;
  }
  family = AF_INET;
  return inet_pton(AF_INET, text.c_str(), buf) == 1;
}

char* formatV4(const unsigned char* b, char* o) {
  for (int i = 0; i < 4; ++i) {
    if (i) *o++ = '.';
    unsigned v = b[i];
    if (v >= 100) *o++ = char('0' + v / 100);
    if (v >= 10) *o++ = char('0' + v / 10 % 10);
    *o++ = char('0' + v % 10);
  }
  return o;
}

// inet_ntop's text, without its per-word sprintf: the longest run (first on
// ties) of >= 2 zero words becomes "::", and ::a.b.c.d / ::ffff:a.b.c.d
// print the embedded IPv4 address (glibc resolv/inet_ntop.c inet_ntop6 --
// the form folly::IPAddressV6::str() returns).
// (into `o`, at most 45 chars; returns the end)
char* formatAddressTo(const unsigned char* raw, int family, char* o) {
  if (family == AF_INET) return formatV4(raw, o);
  unsigned w[8];
  for (int i = 0; i < 8; ++i) w[i] = unsigned(raw[2 * i]) << 8 | raw[2 * i + 1];
  int bestBase = -1, bestLen = 0, curBase = -1, curLen = 0;
  for (int i = 0; i < 8; ++i) {
    if (w[i] == 0) {
      if (curBase < 0) curBase = i, curLen = 1;
      else ++curLen;
    } else if (curBase >= 0) {
      if (bestBase < 0 || curLen > bestLen) bestBase = curBase, bestLen = curLen;
      curBase = -1;
    }
  }
  if (curBase >= 0 && (bestBase < 0 || curLen > bestLen)) bestBase = curBase, bestLen = curLen;
  if (bestBase >= 0 && bestLen < 2) bestBase = -1;
  static const char hexd[] = "0123456789abcdef";
  for (int i = 0; i < 8; ++i) {
    if (bestBase >= 0 && i >= bestBase && i < bestBase + bestLen) {
      if (i == bestBase) *o++ = ':';
      continue;
    }
    if (i) *o++ = ':';
    if (i == 6 && bestBase == 0 && (bestLen == 6 || (bestLen == 5 && w[5] == 0xffff))) {
      return formatV4(raw + 12, o);
    }
    unsigned v = w[i];
    bool lead = true;
    for (int sh = 12; sh >= 0; sh -= 4) {
      unsigned d = (v >> sh) & 0xf;
      if (d || !lead || sh == 0) *o++ = hexd[d], lead = false;
    }
  }
  if (bestBase >= 0 && bestBase + bestLen == 8) *o++ = ':';
  return o;
}

std::string formatAddress(const unsigned char* raw, int family) {
  char buf[48];
  return std::string(buf, formatAddressTo(raw, family, buf));
}

// "<addr>/<len>" in one string construction (len in 0..128)
std::string formatPrefix(const unsigned char* raw, int family, int len) {
  char buf[64];
  char* o = formatAddressTo(raw, family, buf);
  *o++ = '/';
  if (len >= 100) *o++ = char('0' + len / 100);
  if (len >= 10) *o++ = char('0' + len / 10 % 10);
  *o++ = char('0' + len % 10);
  return std::string(buf, o);
}

bool validNodeChar(char c) {  // LsdbTypes.h:452-457 node class
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
         c == '.' || c == '-' || c == '_';
}

bool validIpChar(char c) {
  return (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F') || (c >= '0' && c <= '9') ||
         c == '.' || c == ':';
}

// PrefixKey::fromStr (LsdbTypes.cpp:28-48): "prefix:<node>:[<ip>/<plen>]"
std::optional<std::pair<std::string, std::string>> parsePrefixKey(const std::string& key) {
  static const std::string marker = "prefix:";
  if (key.compare(0, marker.size(), marker) != 0) return std::nullopt;
  size_t i = marker.size(), n = key.size();
  // node is greedy over its class; the class excludes ':' so the first ':'
  // ends it
  size_t b = i;
  while (i < n && validNodeChar(key[i])) ++i;
  if (i == b || i + 1 >= n || key[i] != ':' || key[i + 1] != '[') return std::nullopt;
  std::string node = key.substr(b, i - b);
  i += 2;
  // IPAddr is greedy over [a-fA-F\d.:]+ followed by '/'
  b = i;
  while (i < n && validIpChar(key[i])) ++i;
  if (i == b || i >= n || key[i] != '/') return std::nullopt;
  std::string ip = key.substr(b, i - b);
  ++i;
  b = i;
  while (i < n && key[i] >= '0' && key[i] <= '9') ++i;
  if (i == b || i - b > 3 || i + 1 != n || key[i] != ']') return std::nullopt;
  int plen = std::stoi(key.substr(b, i - b));
  unsigned char buf[16];
  int fam;
  if (!parseAddress(ip, buf, fam)) return std::nullopt;
  std::string raw(reinterpret_cast<char*>(buf), fam == AF_INET6 ? 16 : 4);
  try {
    return std::make_pair(node, ipPrefixToNetworkString(raw, int16_t(plen)));
  } catch (const LsdbDecodeError&) {
    return std::nullopt;
  }
}

}  // namespace

// ------------------------------------------------------------ public --
std::string binaryAddressToString(std::string_view raw) {
  if (raw.empty()) return {};
  if (raw.size() == 4) return formatAddress(reinterpret_cast<const unsigned char*>(raw.data()), AF_INET);
  if (raw.size() == 16) return formatAddress(reinterpret_cast<const unsigned char*>(raw.data()), AF_INET6);
  fail("address: BinaryAddress.addr must be 4 or 16 bytes");  // IPAddress::fromBinary
}

std::string stringToBinaryAddress(const std::string& text) {
  if (text.empty()) return {};
  unsigned char buf[16];
  int fam;
  if (!parseAddress(text, buf, fam)) throw std::invalid_argument("bad IP address: " + text);
  return std::string(reinterpret_cast<char*>(buf), fam == AF_INET6 ? 16 : 4);
}

// The IpPrefix as advertised, "<addr>/<len>" with the host bits kept
// (toString of the raw thrift struct's address, NetworkUtil.h:26-40).
std::string ipPrefixToString(std::string_view raw, int16_t len) {
  if (raw.size() != 4 && raw.size() != 16) fail("prefix: address must be 4 or 16 bytes");
  int bits = int(raw.size()) * 8;
  if (len < 0 || len > bits) fail("prefix: length out of range");
  return formatPrefix(reinterpret_cast<const unsigned char*>(raw.data()),
                      raw.size() == 16 ? AF_INET6 : AF_INET, len);
}

// "<addr>/<len>" text -> toIPNetwork(prefix, applyMask) printed as
// folly::IPAddress::networkToString (NetworkUtil.h:196-208).
std::string prefixNetworkKey(const std::string& text, bool applyMask) {
  auto slash = text.rfind('/');
  if (slash == std::string::npos || slash + 1 == text.size() || text.size() - slash > 4)
    throw std::invalid_argument("Invalid IPAddress: " + text);
  int len = 0;
  for (size_t i = slash + 1; i < text.size(); ++i) {
    if (text[i] < '0' || text[i] > '9') throw std::invalid_argument("Invalid IPAddress: " + text);
    len = len * 10 + (text[i] - '0');
  }
  unsigned char buf[16];
  int fam;
  if (!parseAddress(text.substr(0, slash), buf, fam))
    throw std::invalid_argument("Invalid IPAddress: " + text);
  const int bits = fam == AF_INET6 ? 128 : 32;
  if (len > bits) throw std::invalid_argument("Invalid IPAddress: " + text);
  if (applyMask)
    for (int bit = len; bit < bits; ++bit) buf[bit >> 3] &= uint8_t(~(0x80u >> (bit & 7)));
  return formatPrefix(buf, fam, len);
}

// toIPNetwork(prefix, applyMask=true) (NetworkUtil.h:196-208) printed as
// folly::IPAddress::networkToString: "<masked addr>/<len>"
std::string ipPrefixToNetworkString(std::string_view raw, int16_t len) {
  if (raw.size() != 4 && raw.size() != 16) fail("prefix: address must be 4 or 16 bytes");
  int bits = int(raw.size()) * 8;
  if (len < 0 || len > bits) fail("prefix: length out of range");
  unsigned char buf[16];
  std::memcpy(buf, raw.data(), raw.size());
  for (int bit = len; bit < bits; ++bit) buf[bit >> 3] &= uint8_t(~(0x80u >> (bit & 7)));
  return formatPrefix(buf, raw.size() == 16 ? AF_INET6 : AF_INET, len);
}

AdjacencyDatabase readAdjacencyDatabase(std::string_view bytes) {  // Types.thrift:223-270
  Reader r(bytes);
  AdjacencyDatabase db;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1:
        if (t == CT_BINARY) { db.thisNodeName = r.bytes(); continue; }
        break;
      case 2:
        if (isBoolType(t)) { db.isOverloaded = t == CT_TRUE; continue; }
        break;
      case 3:
        if (t == CT_LIST) {
          auto [et, n] = r.listHeader();
          if (et != CT_STRUCT) {
            for (uint32_t i = 0; i < n; ++i) r.skipElem(et, 1);
            continue;
          }
          db.adjacencies.reserve(n);
          for (uint32_t i = 0; i < n; ++i) db.adjacencies.push_back(readAdjacency(r));
          continue;
        }
        break;
      case 4:
        if (t == CT_I32) { db.nodeLabel = r.zz32(); continue; }
        break;
      case 5:
        if (t == CT_STRUCT) {
          db.perfEvents.emplace();
          readPerfEvents(r, *db.perfEvents);
          continue;
        }
        break;
      case 6:
        if (t == CT_BINARY) { db.area = r.bytes(); continue; }
        break;
      case 7:
        if (t == CT_I32) { db.nodeMetricIncrementVal = r.zz32(); continue; }
        break;
    }
    r.skip(t, 0);
  }
  return db;
}

namespace {
// networks: every entry's toIPNetwork text; first: the first entry's only
// into `db`, reusing its entry vector's storage (the ingestion loop decodes
// every key into one scratch database: no vector allocation per key)
void readPrefixDbInto(PrefixDatabase& db, std::string_view bytes,
                      std::vector<std::string>* networks, std::string* first) {
  Reader r(bytes);
  if (networks) networks->clear();
  db.thisNodeName.clear();
  db.prefixEntries.clear();
  db.perfEvents.reset();
  db.deletePrefix = false;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1:
        if (t == CT_BINARY) { db.thisNodeName = r.bytes(); continue; }
        break;
      case 3:
        if (t == CT_LIST) {
          auto [et, n] = r.listHeader();
          if (et != CT_STRUCT) {
            for (uint32_t i = 0; i < n; ++i) r.skipElem(et, 1);
            continue;
          }
          db.prefixEntries.reserve(n);
          if (networks) networks->resize(db.prefixEntries.size() + n);
          for (uint32_t i = 0; i < n; ++i) {
            std::string* net = networks ? &(*networks)[db.prefixEntries.size()]
                               : (first && db.prefixEntries.empty()) ? first : nullptr;
            db.prefixEntries.push_back(readPrefixEntry(r, net));
          }
          continue;
        }
        break;
      case 4:
        if (t == CT_STRUCT) {
          db.perfEvents.emplace();
          readPerfEvents(r, *db.perfEvents);
          continue;
        }
        break;
      case 5:
        if (isBoolType(t)) { db.deletePrefix = t == CT_TRUE; continue; }
        break;
    }
    r.skip(t, 0);
  }
}

PrefixDatabase readPrefixDb(std::string_view bytes, std::vector<std::string>* networks,
                            std::string* first) {  // Types.thrift:415-430
  PrefixDatabase db;
  readPrefixDbInto(db, bytes, networks, first);
  return db;
}
}  // namespace

PrefixDatabase readPrefixDatabase(std::string_view bytes, std::vector<std::string>* networks) {
  return readPrefixDb(bytes, networks, nullptr);
}

std::string writeAdjacencyDatabase(const AdjacencyDatabase& db) {
  Writer w;
  w.out.reserve(64 + 96 * db.adjacencies.size());
  int16_t l = 0;
  w.field(l, 1, CT_BINARY); w.bytes(db.thisNodeName);
  w.boolField(l, 2, db.isOverloaded);
  w.field(l, 3, CT_LIST);
  w.listHeader(CT_STRUCT, db.adjacencies.size());
  for (const auto& a : db.adjacencies) writeAdjacency(w, a);
  w.field(l, 4, CT_I32); w.zz(db.nodeLabel);
  if (db.perfEvents) { w.field(l, 5, CT_STRUCT); writePerfEvents(w, *db.perfEvents); }
  w.field(l, 6, CT_BINARY); w.bytes(db.area);
  w.field(l, 7, CT_I32); w.zz(db.nodeMetricIncrementVal);
  w.stop();
  return std::move(w.out);
}

std::string writePrefixDatabase(const PrefixDatabase& db) {
  Writer w;
  int16_t l = 0;
  w.field(l, 1, CT_BINARY); w.bytes(db.thisNodeName);
  w.field(l, 3, CT_LIST);
  w.listHeader(CT_STRUCT, db.prefixEntries.size());
  for (const auto& e : db.prefixEntries) writePrefixEntry(w, e);
  if (db.perfEvents) { w.field(l, 4, CT_STRUCT); writePerfEvents(w, *db.perfEvents); }
  w.boolField(l, 5, db.deletePrefix);
  w.stop();
  return std::move(w.out);
}

int64_t getUnixTimeStampMs() {  // Util: system clock, ms since the epoch
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

void addPerfEvent(PerfEvents& events, const std::string& nodeName,
                  const std::string& descr) {  // LsdbUtil.cpp:52-59
  events.push_back(PerfEvent{nodeName, descr, getUnixTimeStampMs()});
}

std::vector<std::string> sprintPerfEvents(const PerfEvents& events) {  // LsdbUtil.cpp:61-82
  std::vector<std::string> out;
  if (events.empty()) return out;
  int64_t recent = events.front().unixTs;
  for (const auto& e : events) {
    const int64_t d = e.unixTs - recent;
    recent = e.unixTs;
    out.push_back("node: " + e.nodeName + ", event: " + e.eventDescr + ", duration: " +
                  std::to_string(d) + "ms, unix-timestamp: " + std::to_string(e.unixTs));
  }
  return out;
}

int64_t getTotalPerfEventsDuration(const PerfEvents& events) {  // LsdbUtil.cpp:84-93
  if (events.empty()) return 0;
  return events.back().unixTs - events.front().unixTs;
}

std::optional<int64_t> getDurationBetweenPerfEvents(const PerfEvents& events,
                                                    const std::string& first,
                                                    const std::string& second,
                                                    std::string* error) {  // LsdbUtil.cpp:95-128
  auto fail = [&](std::string m) -> std::optional<int64_t> {
    if (error) *error = std::move(m);
    return std::nullopt;
  };
  auto it = std::find_if(events.begin(), events.end(),
                         [&](const PerfEvent& e) { return e.eventDescr == first; });
  if (it == events.end()) return fail("Could not find first event: " + first);
  const int64_t t1 = it->unixTs;
  it = std::find_if(it + 1, events.end(),
                    [&](const PerfEvent& e) { return e.eventDescr == second; });
  if (it == events.end()) return fail("Could not find second event: " + second);
  const int64_t t2 = it->unixTs;
  if (t2 < t1) return fail("Negative duration between first and second event");
  return t2 - t1;
}

std::string getNodeNameFromKey(const std::string& key) {  // LsdbUtil.cpp:691-698
  size_t a = key.find(':');
  if (a == std::string::npos) return "";
  size_t b = key.find(':', a + 1);
  return key.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
}

// The pure half of updateKeyInLsdb: decode (no state touched). The
// publication path calls it single-threaded, streamed key by key (decoding
// on host threads first was measured slower, lsdb_codec.h).
LsdbIngest::Decoded LsdbIngest::decodeKey(const std::string& key,
                                          const std::optional<std::string_view>& rawVal) {
  Decoded d;
  decodeKeyInto(d, key, rawVal);
  return d;
}

void LsdbIngest::decodeKeyInto(Decoded& d, const std::string& key,
                               const std::optional<std::string_view>& rawVal) {
  d.kind = Decoded::kNone;
  d.network.clear();
  d.error.clear();
  if (!rawVal) return;  // TTL update (Decision.cpp:716-720)
  try {
    if (key.compare(0, 4, "adj:") == 0) {
      d.adj = readAdjacencyDatabase(*rawVal);
      d.kind = Decoded::kAdj;
      return;
    }
    if (key.compare(0, 7, "prefix:") == 0) {
      readPrefixDbInto(d.prefix, *rawVal, nullptr, &d.network);  // the first entry's network
      d.kind = Decoded::kPrefix;
    }
  } catch (const std::exception& e) {  // Decision.cpp:781-784: log, drop the key
    d.kind = Decoded::kError;
    d.error = "Failed to deserialize info for key " + key + ". Exception: " + e.what();
  }
}

LsdbKeyUpdate LsdbIngest::applyDecoded(const std::string& area, LinkState& areaLinkState,
                                       PrefixState& prefixState, const std::string& key,
                                       Decoded&& d, bool inInitialization,
                                       DecisionPendingUpdates* direct) const {
  LsdbKeyUpdate u;
  if (d.kind == Decoded::kNone) return u;
  if (d.kind == Decoded::kError) {
    u.kind = LsdbKeyUpdate::kError;
    u.error = std::move(d.error);
    return u;
  }
  try {
    if (d.kind == Decoded::kAdj) {
      AdjacencyDatabase& db = d.adj;
      db.area = area;  // Decision.cpp:732
      u.kind = LsdbKeyUpdate::kAdjacency;
      u.nodeName = db.thisNodeName;
      u.perfEvents = std::move(db.perfEvents);  // Decision.cpp:739
      u.linkChange = areaLinkState.updateAdjacencyDatabase(db, area, inInitialization);
      return u;
    }
    PrefixDatabase& db = d.prefix;
    u.nodeName = db.thisNodeName;
    if (db.prefixEntries.size() != 1) {  // Decision.cpp:750-756
      u.kind = LsdbKeyUpdate::kError;
      u.error = "Expecting exactly one entry per prefix key, publication received from " +
                db.thisNodeName;
      return u;
    }
    PrefixEntry& entry = db.prefixEntries.front();
    // self-redistributed route reflection (Decision.cpp:761-769)
    if (db.thisNodeName == myNodeName_ && !entry.area_stack.empty() &&
        areas_.count(entry.area_stack.back())) {
      return u;
    }
    // PrefixKey(node, toIPNetwork(*entry.prefix()), area) (Decision.cpp:772-773);
    // a default IpPrefix (no prefix field) is rejected by toIPNetwork
    if (d.network.empty()) fail("prefix: PrefixEntry without a prefix");
    u.kind = LsdbKeyUpdate::kPrefix;
    // direct: the changed network goes straight into the pending set (the
    // publication path; no per-key vector or copy)
    if (db.deletePrefix) {
      std::string net;
      if (prefixState.deletePrefixInPlace(db.thisNodeName, area, d.network, &net)) {
        if (direct) direct->addUpdatedPrefix(net);
        else u.changedPrefixes.push_back(std::move(net));
      }
    } else {
      const std::string* net = prefixState.updatePrefixInPlace(
          db.thisNodeName, area, std::move(d.network), std::move(entry));
      if (net) {
        if (direct) direct->addUpdatedPrefix(*net);
        else u.changedPrefixes.push_back(*net);
      }
    }
    // the key's count and perf events (Decision.cpp:775-780): only once the
    // update above did not throw, as applyPrefixStateChange runs after
    // updatePrefix / deletePrefix; straight into `direct` on the publication
    // path, else with the update
    if (direct) direct->notePrefixKey(db.perfEvents);
    else u.perfEvents = std::move(db.perfEvents);
  } catch (const std::exception& e) {  // Decision.cpp:781-784: log, drop the key
    u = LsdbKeyUpdate{};
    u.kind = LsdbKeyUpdate::kError;
    u.error = "Failed to deserialize info for key " + key + ". Exception: " + e.what();
  }
  return u;
}

LsdbKeyUpdate LsdbIngest::updateKeyInLsdb(const std::string& area, LinkState& areaLinkState,
                                          PrefixState& prefixState, const std::string& key,
                                          const std::optional<std::string_view>& rawVal,
                                          bool inInitialization) const {
  // one decode scratch per ingesting thread: its containers keep their
  // storage from key to key (applyDecoded moves the entry and the network
  // out; decodeKeyInto resets every field it reads)
  thread_local Decoded scratch;
  decodeKeyInto(scratch, key, rawVal);
  return applyDecoded(area, areaLinkState, prefixState, key, std::move(scratch),
                      inInitialization);
}

LsdbKeyUpdate LsdbIngest::deleteKeyFromLsdb(const std::string& area, LinkState& areaLinkState,
                                            PrefixState& prefixState,
                                            const std::string& key) const {
  LsdbKeyUpdate u;
  if (key.compare(0, 4, "adj:") == 0) {  // Decision.cpp:795-802
    u.kind = LsdbKeyUpdate::kAdjacency;
    u.nodeName = getNodeNameFromKey(key);
    u.linkChange = areaLinkState.deleteAdjacencyDatabase(u.nodeName);
    return u;
  }
  if (key.compare(0, 7, "prefix:") == 0) {  // Decision.cpp:804-818
    auto pk = parsePrefixKey(key);
    if (!pk) {
      u.kind = LsdbKeyUpdate::kError;
      u.error = "Invalid format for key: " + key + ".";
      return u;
    }
    u.kind = LsdbKeyUpdate::kPrefix;
    u.nodeName = pk->first;
    std::string net;
    if (prefixState.deletePrefixInPlace(pk->first, area, pk->second, &net)) {
      u.changedPrefixes.push_back(std::move(net));
    }
  }
  return u;
}

void DecisionPendingUpdates::apply(const LsdbKeyUpdate& u) {
  if (u.kind == LsdbKeyUpdate::kAdjacency) {
    applyLinkStateChange(u.nodeName, u.linkChange, u.perfEvents);
  } else if (u.kind == LsdbKeyUpdate::kPrefix) {
    applyPrefixStateChange(u.changedPrefixes, u.perfEvents);
  }
}

void LsdbIngest::processPublication(const std::string& area, AreaLinkStates& areaLinkStates,
                                    PrefixState& prefixState,
                                    const std::vector<PublicationKeyVal>& keyVals,
                                    const std::vector<std::string>& expiredKeys,
                                    DecisionPendingUpdates& pending,
                                    bool inInitialization) {
  if (area.empty()) throw std::invalid_argument("publication without area");  // CHECK
  auto it = areaLinkStates.find(area);
  if (it == areaLinkStates.end()) {
    it = areaLinkStates.emplace(area, LinkState(area, myNodeName_)).first;
  }
  areas_.clear();
  for (const auto& [a, _] : areaLinkStates) areas_.insert(a);
  LinkState& ls = it->second;
  if (keyVals.empty() && expiredKeys.empty()) return;
  // keys in std::map order (the thrift map's, Decision.cpp:821-846): a
  // sorted index (already sorted publications skip the sort); a repeated
  // key keeps its last value, as the map assignment would
  std::vector<const PublicationKeyVal*> ordered;
  ordered.reserve(keyVals.size());
  for (const auto& kv : keyVals) ordered.push_back(&kv);
  auto less = [](const PublicationKeyVal* a, const PublicationKeyVal* b) { return a->key < b->key; };
  if (!std::is_sorted(ordered.begin(), ordered.end(), less)) {
    std::stable_sort(ordered.begin(), ordered.end(), less);
  }
  size_t prefixKeys = 0;
  for (const auto& kv : keyVals) prefixKeys += kv.key.compare(0, 7, "prefix:") == 0;
  prefixState.reserve(prefixState.prefixes().size() + prefixKeys);
  pending.reserveUpdatedPrefixes(prefixKeys);
  // the publication's prefix keys note themselves into `pending`
  // (applyDecoded's direct path); adjacency keys apply here
  auto take = [&](LsdbKeyUpdate&& u) {
    if (u.kind != LsdbKeyUpdate::kPrefix) pending.apply(u);
  };
  Decoded scratch;  // reused key to key (decodeKeyInto)
  for (size_t i = 0; i < ordered.size(); ++i) {
    if (i + 1 < ordered.size() && ordered[i + 1]->key == ordered[i]->key) continue;
    const PublicationKeyVal* kv = ordered[i];
    std::optional<std::string_view> v;
    if (kv->value) v = *kv->value;
    decodeKeyInto(scratch, kv->key, v);
    take(applyDecoded(area, ls, prefixState, kv->key, std::move(scratch), inInitialization,
                      &pending));
  }
  for (const auto& key : expiredKeys) pending.apply(deleteKeyFromLsdb(area, ls, prefixState, key));
}

}  // namespace openr_amd
