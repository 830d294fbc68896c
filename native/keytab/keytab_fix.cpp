// keytab-fix: rewrites an MIT keytab into the layout Hadoop 3.2.0's keytab reader accepts.
//
// Counterpart of the reference's hdfs `keytab-fix` tool
// (frameworks/hdfs/keytab-fix/src/main/java/com/mesosphere/keytabfix/KeytabFix.java:7, Keytab.java,
// KeytabEntry.java), which every Kerberized hdfs task runs before starting
// (frameworks/hdfs/src/main/dist/svc.yml:75-76: "Fix keytab file due to bug in HDFS version 3.2.0,
// HADOOP-16283"). Hadoop's reader fails on records that carry the optional trailing 32-bit key
// version (what MIT kadmin / ktutil write), so the tool reads every record and writes it back
// without that trailer, grouped by principal, into ./hdfs.keytab.
//
//   keytab-fix <file.keytab>      -> ./hdfs.keytab (exit 0); 1 on a missing argument/file/bad keytab
//
// File format (MIT keytab, all integers big endian):
//   u16 version (0x0502; 0x0501 = principal component count includes the realm, no name type)
//   records: i32 size (< 0: a deleted record, a hole of -size bytes), then
//     u16 component count, counted realm, counted components, u32 name type (0x0502 only),
//     u32 timestamp, u8 kvno, u16 enctype, counted key data, [u32 kvno if >= 4 bytes remain; 0 = none]
//   counted = u16 length + bytes.
// Rewriting follows the reference tool: the 32-bit kvno, when present and non-zero, replaces the
// 8-bit one and is written back truncated to 8 bits; a zero-length principal component is written
// as the text "null" (the reference reads it as a null string); records are grouped by principal
// in order of first appearance (the reference's HashMap order is unspecified); padding after a
// record is skipped. Where the reference tool cannot work this one does the natural thing: holes
// (negative sizes) are skipped instead of misread, a 0x0501 keytab is written as 0x0502 (name type
// KRB5_NT_PRINCIPAL) instead of a 0x0501 marker over 0x0502 records, and a record without key
// data (enctype 0 or empty key) is dropped with a warning instead of failing the whole file.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

namespace {

struct Entry {
  std::string realm;
  std::vector<std::string> components;
  uint32_t name_type = 1;  // KRB5_NT_PRINCIPAL
  uint32_t timestamp = 0;
  uint32_t kvno = 0;
  uint16_t enctype = 0;
  std::string key;
};

struct Reader {
  const std::vector<unsigned char>& b;
  size_t pos;
  size_t end;
  bool ok = true;

  bool need(size_t n) {
    if (!ok || end < pos || end - pos < n) ok = false;
    return ok;
  }
  uint32_t u8() {
    if (!need(1)) return 0;
    return b[pos++];
  }
  uint32_t u16() {
    if (!need(2)) return 0;
    uint32_t v = (uint32_t(b[pos]) << 8) | b[pos + 1];
    pos += 2;
    return v;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t v = (uint32_t(b[pos]) << 24) | (uint32_t(b[pos + 1]) << 16) | (uint32_t(b[pos + 2]) << 8) | b[pos + 3];
    pos += 4;
    return v;
  }
  std::string counted() {
    const uint32_t n = u16();
    if (!need(n)) return std::string();
    std::string s(reinterpret_cast<const char*>(&b[pos]), n);
    pos += n;
    return s;
  }
};

void put16(std::string& o, uint32_t v) {
  o.push_back(char((v >> 8) & 0xFF));
  o.push_back(char(v & 0xFF));
}
void put32(std::string& o, uint32_t v) {
  o.push_back(char((v >> 24) & 0xFF));
  o.push_back(char((v >> 16) & 0xFF));
  o.push_back(char((v >> 8) & 0xFF));
  o.push_back(char(v & 0xFF));
}
void put_counted(std::string& o, const std::string& s) {
  put16(o, uint32_t(s.size()));
  o += s;
}

std::string principal_key(const Entry& e) {
  std::string k = e.realm;
  for (const auto& c : e.components) k += '\x1f' + c;
  return k;
}

std::string encode(const Entry& e) {
  std::string body;
  put16(body, uint32_t(e.components.size()));
  put_counted(body, e.realm);
  for (const auto& c : e.components) put_counted(body, c.empty() ? std::string("null") : c);
  put32(body, e.name_type);
  put32(body, e.timestamp);
  body.push_back(char(e.kvno & 0xFF));
  put16(body, e.enctype);
  put_counted(body, e.key);
  std::string rec;
  put32(rec, uint32_t(body.size()));
  return rec + body;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "Keytab File is not specified!\nUsage: keytab-fix file.keytab\n");
    return 1;
  }
  const std::string in_path = argv[1];
  const std::string out_path = argc > 2 ? argv[2] : "hdfs.keytab";  // the reference always writes ./hdfs.keytab
  std::ifstream in(in_path, std::ios::binary);
  if (!in) {
    std::fprintf(stderr, "Keytab File does not exists: %s\n", in_path.c_str());
    return 1;
  }
  std::printf("Fixing KeyTab File...%s\n", in_path.c_str());
  std::vector<unsigned char> data((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  Reader r{data, 0, data.size()};
  const uint32_t version = r.u16();
  if (!r.ok || (version != 0x0501 && version != 0x0502)) {
    std::fprintf(stderr, "Not a keytab (version 0x%04x): %s\n", version, in_path.c_str());
    return 1;
  }
  std::vector<std::string> order;                        // principals, first appearance
  std::map<std::string, std::vector<Entry>> by_principal;
  size_t dropped = 0;
  while (r.ok && r.pos < data.size()) {
    if (data.size() - r.pos < 4) break;                  // trailing zero padding shorter than a size
    const int32_t size = int32_t(r.u32());
    if (size == 0) break;                                // MIT: a zero size ends the file
    if (size < 0) {                                      // a deleted record: skip the hole
      const size_t hole = size_t(-int64_t(size));
      if (data.size() - r.pos < hole) {
        r.ok = false;
        break;
      }
      r.pos += hole;
      continue;
    }
    const size_t start = r.pos, rec_end = r.pos + size_t(size);
    if (rec_end > data.size()) {
      std::fprintf(stderr, "Bad keytab: record of %d bytes runs past the end of %s\n", size, in_path.c_str());
      return 1;
    }
    Reader rec{data, start, rec_end};
    Entry e;
    uint32_t n = rec.u16();
    if (version == 0x0501 && n > 0) n -= 1;
    e.realm = rec.counted();
    for (uint32_t i = 0; i < n && rec.ok; ++i) e.components.push_back(rec.counted());
    if (version == 0x0502) e.name_type = rec.u32();
    e.timestamp = rec.u32();
    e.kvno = rec.u8();
    e.enctype = uint16_t(rec.u16());
    e.key = rec.counted();
    if (!rec.ok) {
      std::fprintf(stderr, "Bad keytab: truncated record at offset %zu of %s\n", start - 4, in_path.c_str());
      return 1;
    }
    if (rec_end - rec.pos >= 4) {
      const uint32_t kvno32 = rec.u32();
      if (kvno32 != 0) e.kvno = kvno32;
    }
    r.pos = rec_end;                                     // skip padding inside the record
    if (e.enctype == 0 || e.key.empty()) {
      ++dropped;
      continue;
    }
    const std::string pk = principal_key(e);
    if (by_principal.find(pk) == by_principal.end()) order.push_back(pk);
    by_principal[pk].push_back(e);
  }
  if (!r.ok) {
    std::fprintf(stderr, "Bad keytab: %s is truncated\n", in_path.c_str());
    return 1;
  }
  std::string out;
  put16(out, 0x0502);
  size_t written = 0;
  for (const auto& pk : order) {
    for (const auto& e : by_principal[pk]) {
      out += encode(e);
      ++written;
    }
  }
  std::ofstream o(out_path, std::ios::binary | std::ios::trunc);
  o.write(out.data(), std::streamsize(out.size()));
  if (!o) {
    std::fprintf(stderr, "Cannot write %s\n", out_path.c_str());
    return 1;
  }
  if (dropped != 0) std::fprintf(stderr, "keytab-fix: dropped %zu record(s) without key data\n", dropped);
  std::printf("Fixed KeyTab File is: %s (%zu entries)\n", out_path.c_str(), written);
  return 0;
}
