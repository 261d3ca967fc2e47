// TensorFlow V2 checkpoint (TensorBundle) writer/reader, no TensorFlow dependency.
//
// Layout written (what tf.train.Saver V2 produces):
//   <prefix>.data-00000-of-00001   raw little-endian tensor bytes, concatenated
//   <prefix>.index                 LevelDB-format SSTable: key "" -> BundleHeaderProto,
//                                  key <tensor name> -> BundleEntryProto{dtype, shape, shard_id,
//                                  offset, size, crc32c (masked)}; keys sorted.
// SSTable: data blocks with prefix-compressed entries + restart array, 5-byte trailer
// (compression type 0 + masked crc32c), empty meta-index block, index block (restart interval 1),
// 48-byte footer ending in magic 0xdb4775248b80fb57.
// The reader parses any such table (multiple data shards via shard_id supported).
// Partitioned variables (tf.fixed_size_partitioner under a partitioned variable_scope, e.g. the
// reference's 'partitioned_space' / 'root' trainers) are stored the way TF's BundleWriter::AddSlice
// lays them out: a data-less full-tensor entry {dtype, full shape, slices: [TensorSliceProto]} plus
// one ordinary entry per slice whose key is checkpoint::EncodeTensorNameSlice(name, slice) - an
// OrderedCode string (0, name, rank, (start, length) per dim; binary, so it sorts before every
// plain name).  The writer emits that layout (dtm_bundle_writer_add_slice) and the reader
// reassembles a sliced variable into its full tensor (dtm_bundle_reader_read).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "crc32c.h"

#define API extern "C" __attribute__((visibility("default")))

namespace dtmrt {
namespace {

void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)(v | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}
void put_fixed32(std::string* s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s->push_back((char)((v >> (8 * i)) & 0xff));
}
bool get_varint(const char*& p, const char* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    uint8_t b = (uint8_t)*p++;
    r |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}
uint32_t get_fixed32(const char* p) {
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) v |= (uint32_t)(uint8_t)p[i] << (8 * i);
  return v;
}

// protobuf helpers
void pb_varint(std::string* s, int field, uint64_t v) {
  put_varint(s, ((uint64_t)field << 3) | 0);
  put_varint(s, v);
}
void pb_bytes(std::string* s, int field, const std::string& b) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, b.size());
  s->append(b);
}
void pb_fixed32(std::string* s, int field, uint32_t v) {
  put_varint(s, ((uint64_t)field << 3) | 5);
  put_fixed32(s, v);
}

// one TensorSliceProto: per dim (start, length); length -1 = the full extent
typedef std::vector<std::pair<int64_t, int64_t>> Slice;

struct Entry {
  std::string name;
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;  // masked
  bool sliced = false;
  std::vector<Slice> slices;  // full-tensor entry of a partitioned variable
};

// ---- tensorflow::strings::OrderedCode (the slice-entry key encoding) ------------------------
void oc_num_increasing(std::string* s, uint64_t v) {
  unsigned char buf[8];
  int len = 0;
  while (v) {
    buf[7 - len] = (unsigned char)(v & 0xff);
    v >>= 8;
    ++len;
  }
  s->push_back((char)len);
  s->append((const char*)buf + 8 - len, (size_t)len);
}
void oc_string(std::string* s, const std::string& str) {
  for (unsigned char c : str) {
    if (c == 0x00) { s->push_back('\x00'); s->push_back('\xff'); }
    else if (c == 0xff) { s->push_back('\xff'); s->push_back('\x00'); }
    else s->push_back((char)c);
  }
  s->push_back('\x00');
  s->push_back('\x01');
}
void oc_signed_num_increasing(std::string* s, int64_t val) {
  const uint64_t x = val < 0 ? ~(uint64_t)val : (uint64_t)val;
  if (x < 64) {
    s->push_back((char)(0x80 ^ (uint8_t)val));
    return;
  }
  static const uint8_t hdr[11][2] = {{0, 0},    {0x80, 0}, {0xc0, 0}, {0xe0, 0},    {0xf0, 0},   {0xf8, 0},
                                     {0xfc, 0}, {0xfe, 0}, {0xff, 0}, {0xff, 0x80}, {0xff, 0xc0}};
  const int bits = 64 - __builtin_clzll(x);
  const int len = bits / 7 + 1;
  uint8_t buf[10];
  buf[0] = buf[1] = val < 0 ? 0xff : 0x00;
  for (int i = 0; i < 8; ++i) buf[2 + i] = (uint8_t)((uint64_t)val >> (56 - 8 * i));
  uint8_t* b = buf + 10 - len;
  b[0] ^= hdr[len][0];
  b[1] ^= hdr[len][1];
  s->append((const char*)b, (size_t)len);
}
// checkpoint::EncodeTensorNameSlice
std::string slice_key(const std::string& name, const Slice& sl) {
  std::string k;
  oc_num_increasing(&k, 0);
  oc_string(&k, name);
  oc_num_increasing(&k, sl.size());
  for (const auto& e : sl) {
    oc_signed_num_increasing(&k, e.first);
    oc_signed_num_increasing(&k, e.second);
  }
  return k;
}

std::string encode_entry(const Entry& e) {
  std::string s, shp;
  pb_varint(&s, 1, (uint64_t)e.dtype);
  for (int64_t d : e.shape) {
    std::string dim;
    pb_varint(&dim, 1, (uint64_t)d);
    pb_bytes(&shp, 2, dim);
  }
  pb_bytes(&s, 2, shp);  // TensorShapeProto (present even for scalars)
  if (!e.slices.empty()) {
    // full-tensor entry of a partitioned variable: no shard / offset / size / crc (BundleWriter::AddSlice)
    for (const Slice& sl : e.slices) {
      std::string sp;
      for (const auto& ext : sl) {
        std::string ex;  // TensorSliceProto.Extent: a full extent is an empty message
        if (ext.second >= 0) {
          if (ext.first) pb_varint(&ex, 1, (uint64_t)ext.first);
          pb_varint(&ex, 2, (uint64_t)ext.second);
        }
        pb_bytes(&sp, 1, ex);
      }
      pb_bytes(&s, 7, sp);
    }
    return s;
  }
  if (e.shard) pb_varint(&s, 3, (uint64_t)e.shard);
  if (e.offset) pb_varint(&s, 4, (uint64_t)e.offset);
  if (e.size) pb_varint(&s, 5, (uint64_t)e.size);
  pb_fixed32(&s, 6, e.crc);
  return s;
}

bool skip_field(const char*& p, const char* end, int wt);

bool decode_slice(const char* p, const char* end, Slice* sl) {
  while (p < end) {
    uint64_t key, len;
    if (!get_varint(p, end, &key)) return false;
    if ((key >> 3) == 1 && (key & 7) == 2) {
      if (!get_varint(p, end, &len) || p + len > end) return false;
      const char* q = p, *qe = p + len;
      int64_t start = 0, length = -1;
      while (q < qe) {
        uint64_t k2, v2;
        if (!get_varint(q, qe, &k2)) return false;
        if ((k2 & 7) == 0) {
          if (!get_varint(q, qe, &v2)) return false;
          if ((k2 >> 3) == 1) start = (int64_t)v2;
          else if ((k2 >> 3) == 2) length = (int64_t)v2;
        } else if (!skip_field(q, qe, (int)(k2 & 7))) {
          return false;
        }
      }
      sl->emplace_back(start, length);
      p = qe;
    } else if (!skip_field(p, end, (int)(key & 7))) {
      return false;
    }
  }
  return true;
}

std::string encode_header(int num_shards) {
  std::string s, ver;
  pb_varint(&s, 1, (uint64_t)num_shards);
  // endianness LITTLE = 0 (default, omitted); version {producer: 1}
  pb_varint(&ver, 1, 1);
  pb_bytes(&s, 3, ver);
  return s;
}

bool skip_field(const char*& p, const char* end, int wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, end, &v);
    case 1: p += 8; return p <= end;
    case 2: if (!get_varint(p, end, &v)) return false; p += v; return p <= end;
    case 5: p += 4; return p <= end;
    default: return false;
  }
}

bool decode_shape(const char* p, const char* end, std::vector<int64_t>* shape) {
  while (p < end) {
    uint64_t key, len;
    if (!get_varint(p, end, &key)) return false;
    int f = (int)(key >> 3), wt = (int)(key & 7);
    if (f == 2 && wt == 2) {
      if (!get_varint(p, end, &len)) return false;
      const char* q = p, *qe = p + len;
      int64_t size = 0;
      while (q < qe) {
        uint64_t k2, v2;
        if (!get_varint(q, qe, &k2)) return false;
        if ((k2 >> 3) == 1 && (k2 & 7) == 0) {
          if (!get_varint(q, qe, &v2)) return false;
          size = (int64_t)v2;
        } else if (!skip_field(q, qe, (int)(k2 & 7))) {
          return false;
        }
      }
      shape->push_back(size);
      p = qe;
    } else if (!skip_field(p, end, wt)) {
      return false;
    }
  }
  return true;
}

bool decode_entry(const std::string& val, Entry* e) {
  const char* p = val.data();
  const char* end = p + val.size();
  while (p < end) {
    uint64_t key, v;
    if (!get_varint(p, end, &key)) return false;
    int f = (int)(key >> 3), wt = (int)(key & 7);
    if (wt == 0) {
      if (!get_varint(p, end, &v)) return false;
      if (f == 1) e->dtype = (int)v;
      else if (f == 3) e->shard = (int)v;
      else if (f == 4) e->offset = (int64_t)v;
      else if (f == 5) e->size = (int64_t)v;
    } else if (wt == 5) {
      if (p + 4 > end) return false;
      if (f == 6) e->crc = get_fixed32(p);
      p += 4;
    } else if (wt == 2) {
      if (!get_varint(p, end, &v)) return false;
      if (f == 2) {
        if (!decode_shape(p, p + v, &e->shape)) return false;
      } else if (f == 7) {
        e->sliced = true;
        Slice sl;
        if (!decode_slice(p, p + v, &sl)) return false;
        e->slices.push_back(sl);
      }
      p += v;
    } else if (!skip_field(p, end, wt)) {
      return false;
    }
  }
  return true;
}

// ---- SSTable builder -----------------------------------------------------------------------
class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      size_t n = std::min(last_key_.size(), key.size());
      while (shared < n && last_key_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back((uint32_t)buf_.size());
      counter_ = 0;
    }
    put_varint(&buf_, shared);
    put_varint(&buf_, key.size() - shared);
    put_varint(&buf_, value.size());
    buf_.append(key.data() + shared, key.size() - shared);
    buf_.append(value);
    last_key_ = key;
    ++counter_;
  }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) put_fixed32(&out, r);
    put_fixed32(&out, (uint32_t)restarts_.size());
    return out;
  }
  size_t size_estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return buf_.empty(); }
  void reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    last_key_.clear();
  }

 private:
  int interval_;
  int counter_ = 0;
  std::string buf_, last_key_;
  std::vector<uint32_t> restarts_;
};

void write_block(std::string* file, const std::string& contents, uint64_t* off, uint64_t* size) {
  *off = file->size();
  *size = contents.size();
  file->append(contents);
  char type = 0;
  uint32_t crc = crc32c_extend(crc32c(contents.data(), contents.size()), &type, 1);
  file->push_back(type);
  put_fixed32(file, crc_mask(crc));
}

std::string build_table(const std::vector<std::pair<std::string, std::string>>& kv) {
  std::string file;
  BlockBuilder data(16), index(1);
  std::string last_key;
  auto flush = [&]() {
    if (data.empty()) return;
    uint64_t off, size;
    write_block(&file, data.finish(), &off, &size);
    std::string handle;
    put_varint(&handle, off);
    put_varint(&handle, size);
    index.add(last_key, handle);
    data.reset();
  };
  for (const auto& e : kv) {
    data.add(e.first, e.second);
    last_key = e.first;
    if (data.size_estimate() >= 4096) flush();
  }
  flush();
  BlockBuilder meta(16);
  uint64_t moff, msize, ioff, isize;
  write_block(&file, meta.finish(), &moff, &msize);
  write_block(&file, index.finish(), &ioff, &isize);
  std::string footer;
  put_varint(&footer, moff);
  put_varint(&footer, msize);
  put_varint(&footer, ioff);
  put_varint(&footer, isize);
  footer.resize(40, '\0');
  const uint64_t magic = 0xdb4775248b80fb57ull;
  put_fixed32(&footer, (uint32_t)(magic & 0xffffffffu));
  put_fixed32(&footer, (uint32_t)(magic >> 32));
  file.append(footer);
  return file;
}

// ---- SSTable reader -------------------------------------------------------------------------
bool read_file(const std::string& path, std::string* out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out->resize((size_t)n);
  bool ok = n == 0 || std::fread(&(*out)[0], 1, (size_t)n, f) == (size_t)n;
  std::fclose(f);
  return ok;
}

bool parse_block(const std::string& file, uint64_t off, uint64_t size,
                 std::vector<std::pair<std::string, std::string>>* out) {
  if (off + size + 5 > file.size() || size < 4) return false;
  const char* base = file.data() + off;
  // verify trailer crc
  uint32_t stored = crc_unmask(get_fixed32(base + size + 1));
  uint32_t crc = crc32c_extend(crc32c(base, size), base + size, 1);
  if (stored != crc) return false;
  if (base[size] != 0) return false;  // compressed blocks unsupported
  uint32_t nrest = get_fixed32(base + size - 4);
  if ((uint64_t)nrest * 4 + 4 > size) return false;
  const char* p = base;
  const char* end = base + size - 4 - 4 * nrest;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, &shared) || !get_varint(p, end, &nonshared) || !get_varint(p, end, &vlen)) return false;
    if (p + nonshared + vlen > end || shared > key.size()) return false;
    key.resize(shared);
    key.append(p, nonshared);
    p += nonshared;
    out->emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
  return true;
}

bool parse_table(const std::string& file, std::vector<std::pair<std::string, std::string>>* kv) {
  if (file.size() < 48) return false;
  const char* f = file.data() + file.size() - 48;
  uint64_t magic = (uint64_t)get_fixed32(f + 40) | ((uint64_t)get_fixed32(f + 44) << 32);
  if (magic != 0xdb4775248b80fb57ull) return false;
  const char* p = f;
  uint64_t moff, msize, ioff, isize;
  if (!get_varint(p, f + 40, &moff) || !get_varint(p, f + 40, &msize) || !get_varint(p, f + 40, &ioff) ||
      !get_varint(p, f + 40, &isize))
    return false;
  std::vector<std::pair<std::string, std::string>> index;
  if (!parse_block(file, ioff, isize, &index)) return false;
  for (auto& ie : index) {
    const char* q = ie.second.data();
    uint64_t boff, bsize;
    if (!get_varint(q, q + ie.second.size(), &boff) || !get_varint(q, q + ie.second.size(), &bsize)) return false;
    if (!parse_block(file, boff, bsize, kv)) return false;
  }
  return true;
}

struct Writer {
  std::string prefix;
  FILE* data = nullptr;
  int64_t off = 0;
  std::vector<Entry> entries;
  std::map<std::string, Entry> full;  // partitioned variables: name -> full-tensor entry
};

struct Reader {
  std::string prefix;
  int num_shards = 1;
  std::vector<Entry> entries;               // plain tensors + full entries of partitioned ones
  std::map<std::string, Entry> slice_entries;  // encoded slice key -> entry
  std::map<int, FILE*> shards;
  ~Reader() {
    for (auto& s : shards) std::fclose(s.second);
  }
};

std::string shard_name(const std::string& prefix, int i, int n) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), ".data-%05d-of-%05d", i, n);
  return prefix + buf;
}
}  // namespace
}  // namespace dtmrt

using namespace dtmrt;

API void* dtm_bundle_writer_new(const char* prefix) {
  Writer* w = new Writer();
  w->prefix = prefix;
  w->data = std::fopen((w->prefix + ".data-00000-of-00001.tempstate").c_str(), "wb");
  if (!w->data) {
    delete w;
    return nullptr;
  }
  return w;
}

// (the key is a std::string: an encoded slice key contains NUL bytes)
static int writer_add(Writer* w, const std::string& name, int dtype, const int64_t* shape, int ndim, const void* data,
                      int64_t nbytes) {
  Entry e;
  e.name = name;
  e.dtype = dtype;
  e.shape.assign(shape, shape + ndim);
  e.offset = w->off;
  e.size = nbytes;
  e.crc = crc_mask(crc32c(data, (size_t)nbytes));
  if (nbytes && std::fwrite(data, 1, (size_t)nbytes, w->data) != (size_t)nbytes) return -1;
  w->off += nbytes;
  w->entries.push_back(e);
  return 0;
}

API int dtm_bundle_writer_add(void* h, const char* name, int dtype, const int64_t* shape, int ndim, const void* data,
                              int64_t nbytes) {
  return writer_add((Writer*)h, name, dtype, shape, ndim, data, nbytes);
}

// One slice of a partitioned variable: starts/lengths per dim of the FULL tensor (length -1 = full
// extent), data = the slice's values (C order, shape = the lengths).
API int dtm_bundle_writer_add_slice(void* h, const char* name, int dtype, const int64_t* full_shape, int ndim,
                                    const int64_t* starts, const int64_t* lengths, const void* data, int64_t nbytes) {
  Writer* w = (Writer*)h;
  Slice sl;
  std::vector<int64_t> sshape;
  for (int d = 0; d < ndim; ++d) {
    if (starts[d] < 0 || (lengths[d] >= 0 && starts[d] + lengths[d] > full_shape[d])) return -4;
    sl.emplace_back(starts[d], lengths[d]);
    sshape.push_back(lengths[d] < 0 ? full_shape[d] : lengths[d]);
  }
  Entry& f = w->full[name];
  if (f.name.empty()) {
    f.name = name;
    f.dtype = dtype;
    f.shape.assign(full_shape, full_shape + ndim);
  } else if (f.dtype != dtype || f.shape != std::vector<int64_t>(full_shape, full_shape + ndim)) {
    return -5;
  }
  f.slices.push_back(sl);
  const std::string key = slice_key(name, sl);
  return writer_add(w, key, dtype, sshape.data(), ndim, data, nbytes) == 0 ? 0 : -1;
}

API int dtm_bundle_writer_finish(void* h) {
  Writer* w = (Writer*)h;
  int rc = 0;
  for (auto& kv : w->full) w->entries.push_back(kv.second);
  if (std::fclose(w->data) != 0) rc = -1;
  std::sort(w->entries.begin(), w->entries.end(), [](const Entry& a, const Entry& b) { return a.name < b.name; });
  for (size_t i = 1; i < w->entries.size(); ++i)
    if (w->entries[i].name == w->entries[i - 1].name) rc = -3;  // duplicate key
  std::vector<std::pair<std::string, std::string>> kv;
  kv.emplace_back("", encode_header(1));
  for (auto& e : w->entries) kv.emplace_back(e.name, encode_entry(e));
  std::string table = build_table(kv);
  std::string ipath = w->prefix + ".index";
  FILE* f = std::fopen((ipath + ".tempstate").c_str(), "wb");
  if (!f) rc = -1;
  else {
    if (std::fwrite(table.data(), 1, table.size(), f) != table.size()) rc = -1;
    if (std::fclose(f) != 0) rc = -1;
  }
  if (rc == 0) {
    if (std::rename((w->prefix + ".data-00000-of-00001.tempstate").c_str(),
                    (w->prefix + ".data-00000-of-00001").c_str()) != 0 ||
        std::rename((ipath + ".tempstate").c_str(), ipath.c_str()) != 0)
      rc = -2;
  }
  delete w;
  return rc;
}

API void* dtm_bundle_reader_open(const char* prefix) {
  std::string file;
  Reader* r = new Reader();
  r->prefix = prefix;
  if (!read_file(r->prefix + ".index", &file)) {
    delete r;
    return nullptr;
  }
  std::vector<std::pair<std::string, std::string>> kv;
  if (!parse_table(file, &kv)) {
    delete r;
    return nullptr;
  }
  for (auto& p : kv) {
    if (p.first.empty()) {  // header
      const char* q = p.second.data();
      const char* end = q + p.second.size();
      while (q < end) {
        uint64_t key, v;
        if (!get_varint(q, end, &key)) break;
        if ((key >> 3) == 1 && (key & 7) == 0) {
          get_varint(q, end, &v);
          r->num_shards = (int)v;
        } else if (!skip_field(q, end, (int)(key & 7))) {
          break;
        }
      }
      continue;
    }
    Entry e;
    e.name = p.first;
    if (!decode_entry(p.second, &e)) {
      delete r;
      return nullptr;
    }
    if (e.name[0] == '\0') r->slice_entries[e.name] = e;  // an EncodeTensorNameSlice key
    else r->entries.push_back(e);
  }
  return r;
}

API int dtm_bundle_reader_num(void* h) { return (int)((Reader*)h)->entries.size(); }
API const char* dtm_bundle_reader_name(void* h, int i) { return ((Reader*)h)->entries[i].name.c_str(); }

static int dtype_size(int dt) {
  switch (dt) {
    case 1: case 3: return 4;          // float, int32
    case 2: case 9: return 8;          // double, int64
    case 4: case 6: case 10: return 1; // uint8, int8, bool
    case 5: case 14: case 17: case 19: return 2;  // int16, bfloat16, uint16, half
    default: return 0;
  }
}

static int64_t full_bytes(const Entry& e) {
  int64_t n = dtype_size(e.dtype);
  for (int64_t d : e.shape) n *= d;
  return n;
}

// sliced: 1 when the entry is a partitioned variable (read reassembles its slices), nbytes = full size
API int dtm_bundle_reader_info2(void* h, int i, int* dtype, int64_t* shape, int* ndim, int64_t* nbytes, int* sliced) {
  Reader* r = (Reader*)h;
  if (i < 0 || i >= (int)r->entries.size()) return -1;
  const Entry& e = r->entries[i];
  *dtype = e.dtype;
  *ndim = (int)std::min<size_t>(e.shape.size(), 8);
  for (int d = 0; d < *ndim; ++d) shape[d] = e.shape[d];
  *nbytes = e.sliced ? full_bytes(e) : e.size;
  *sliced = e.sliced ? 1 : 0;
  return 0;
}

API int dtm_bundle_reader_info(void* h, int i, int* dtype, int64_t* shape, int* ndim, int64_t* nbytes) {
  int sliced = 0;
  return dtm_bundle_reader_info2(h, i, dtype, shape, ndim, nbytes, &sliced);
}

static int read_entry(Reader* r, const Entry& e, void* dst, int64_t nbytes);

// reassemble a partitioned variable: every slice's data is copied into its box of the full tensor
static int read_sliced(Reader* r, const Entry& e, void* dst, int64_t nbytes) {
  const int es = dtype_size(e.dtype), nd = (int)e.shape.size();
  if (!es || nbytes != full_bytes(e)) return -1;
  std::vector<int64_t> fstride(nd + 1, 1);
  for (int d = nd - 1; d >= 0; --d) fstride[d] = fstride[d + 1] * e.shape[d];
  int64_t covered = 0;
  for (const Slice& sl : e.slices) {
    if ((int)sl.size() != nd) return -4;
    std::vector<int64_t> st(nd), ln(nd);
    int64_t cnt = 1;
    for (int d = 0; d < nd; ++d) {
      st[d] = sl[d].first;
      ln[d] = sl[d].second < 0 ? e.shape[d] : sl[d].second;
      if (st[d] < 0 || st[d] + ln[d] > e.shape[d]) return -4;
      cnt *= ln[d];
    }
    auto it = r->slice_entries.find(slice_key(e.name, sl));
    if (it == r->slice_entries.end() || it->second.size != cnt * es) return -4;
    std::vector<char> buf((size_t)(cnt * es));
    int rc = read_entry(r, it->second, buf.data(), (int64_t)buf.size());
    if (rc) return rc;
    covered += cnt;
    if (cnt == 0) continue;
    // copy rows of the innermost dim: iterate the outer index tuple of the slice box
    const int64_t row = (nd ? ln[nd - 1] : 1) * es;
    const int64_t rows = nd ? cnt / ln[nd - 1] : 1;
    std::vector<int64_t> idx(nd, 0);
    for (int64_t rrow = 0; rrow < rows; ++rrow) {
      int64_t off = 0;
      for (int d = 0; d < nd; ++d) off += (st[d] + idx[d]) * fstride[d + 1];
      std::memcpy((char*)dst + off * es, buf.data() + rrow * row, (size_t)row);
      for (int d = nd - 2; d >= 0; --d) {  // odometer over the outer dims
        if (++idx[d] < ln[d]) break;
        idx[d] = 0;
      }
    }
  }
  int64_t total = 1;
  for (int64_t d : e.shape) total *= d;
  return covered == total ? 0 : -4;  // slices must tile the tensor (TF partitions do, disjointly)
}

API int dtm_bundle_reader_read(void* h, int i, void* dst, int64_t nbytes) {
  Reader* r = (Reader*)h;
  if (i < 0 || i >= (int)r->entries.size()) return -1;
  const Entry& e = r->entries[i];
  if (e.sliced) return read_sliced(r, e, dst, nbytes);
  return read_entry(r, e, dst, nbytes);
}

static int read_entry(Reader* r, const Entry& e, void* dst, int64_t nbytes) {
  if (nbytes != e.size) return -1;
  FILE*& f = r->shards[e.shard];
  if (!f) {
    f = std::fopen(shard_name(r->prefix, e.shard, r->num_shards).c_str(), "rb");
    if (!f) return -3;
  }
  if (std::fseek(f, (long)e.offset, SEEK_SET) != 0) return -3;
  if (nbytes && std::fread(dst, 1, (size_t)nbytes, f) != (size_t)nbytes) return -3;
  if (crc_mask(crc32c(dst, (size_t)nbytes)) != e.crc) return -2;
  return 0;
}

API void dtm_bundle_reader_close(void* h) { delete (Reader*)h; }
