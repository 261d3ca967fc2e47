// Host-side data runtime (replaces TF's FixedLengthRecordReader / TFRecordReader / queue runners;
// SURVEY.md §2.8 C45/C47, K20):
//   * TFRecord framing reader/writer (uint64 length, masked crc32c of length, payload, masked crc32c)
//   * CIFAR-10 binary reader (1 label byte + 3072 CHW bytes per record) into an in-memory HWC table
//   * a prefetching batch loader: a C++ worker thread samples (optionally shuffled) records and
//     fills caller-owned (pinned) host slots in a ring; Python copies a ready slot to the GPU and
//     releases it.  Augmentation runs on the GPU (ops/image.py), not here.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "crc32c.h"

#define API extern "C" __attribute__((visibility("default")))

using namespace dtmrt;

// ---------------------------------------------------------------------------------------------
// TFRecord
namespace {
struct TFRecordReader {
  FILE* f = nullptr;
  std::vector<char> buf;
  bool verify = true;
};
}  // namespace

API void* dtm_tfrecord_writer_open(const char* path) { return std::fopen(path, "wb"); }

API int dtm_tfrecord_write(void* h, const void* data, int64_t n) {
  FILE* f = (FILE*)h;
  uint64_t len = (uint64_t)n;
  char hdr[12];
  std::memcpy(hdr, &len, 8);
  uint32_t lc = crc_mask(crc32c(hdr, 8));
  std::memcpy(hdr + 8, &lc, 4);
  uint32_t dc = crc_mask(crc32c(data, (size_t)n));
  if (std::fwrite(hdr, 1, 12, f) != 12) return -1;
  if (n && std::fwrite(data, 1, (size_t)n, f) != (size_t)n) return -1;
  if (std::fwrite(&dc, 1, 4, f) != 4) return -1;
  return 0;
}

API int dtm_tfrecord_writer_close(void* h) { return std::fclose((FILE*)h) == 0 ? 0 : -1; }

API void* dtm_tfrecord_reader_open(const char* path, int verify) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return nullptr;
  TFRecordReader* r = new TFRecordReader();
  r->f = f;
  r->verify = verify != 0;
  return r;
}

// returns payload length, -1 at EOF, -2 on corruption; *data points into an internal buffer
API int64_t dtm_tfrecord_next(void* h, const char** data) {
  TFRecordReader* r = (TFRecordReader*)h;
  char hdr[12];
  size_t got = std::fread(hdr, 1, 12, r->f);
  if (got == 0) return -1;
  if (got != 12) return -2;
  uint64_t len;
  uint32_t lc;
  std::memcpy(&len, hdr, 8);
  std::memcpy(&lc, hdr + 8, 4);
  if (r->verify && crc_mask(crc32c(hdr, 8)) != lc) return -2;
  if (len > (1ull << 34)) return -2;
  r->buf.resize(len + 4);
  if (std::fread(r->buf.data(), 1, len + 4, r->f) != len + 4) return -2;
  uint32_t dc;
  std::memcpy(&dc, r->buf.data() + len, 4);
  if (r->verify && crc_mask(crc32c(r->buf.data(), len)) != dc) return -2;
  *data = r->buf.data();
  return (int64_t)len;
}

API void dtm_tfrecord_reader_close(void* h) {
  TFRecordReader* r = (TFRecordReader*)h;
  std::fclose(r->f);
  delete r;
}

// ---------------------------------------------------------------------------------------------
// CIFAR-10 binary + prefetching loader
namespace {
struct Table {
  int H = 32, W = 32, C = 3;
  std::vector<uint8_t> images;  // N x H x W x C (HWC)
  std::vector<int32_t> labels;
  size_t n() const { return labels.size(); }
};

struct Loader {
  Table table;
  int batch = 0;
  int nslots = 0;
  std::vector<uint8_t*> img_slots;
  std::vector<int32_t*> lab_slots;
  std::vector<int> state;  // 0 free, 1 filling, 2 ready
  int next_fill = 0, next_get = 0;
  bool shuffle = true;
  uint64_t seed = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<bool> stop{false};
  std::thread worker;
  std::vector<uint32_t> perm;
  size_t cursor = 0;
  std::mt19937_64 rng;
};

bool load_cifar_file(const char* path, int label_bytes, Table* t) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  const int rec = label_bytes + 3072;
  std::vector<uint8_t> buf(rec);
  while (std::fread(buf.data(), 1, rec, f) == (size_t)rec) {
    t->labels.push_back(buf[label_bytes - 1]);  // CIFAR-100 binary: coarse, fine -> use fine
    size_t base = t->images.size();
    t->images.resize(base + 3072);
    const uint8_t* chw = buf.data() + label_bytes;
    uint8_t* hwc = t->images.data() + base;
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < 1024; ++i) hwc[i * 3 + c] = chw[c * 1024 + i];
  }
  std::fclose(f);
  return true;
}

void fill(Loader* L, int slot) {
  const size_t per = (size_t)L->table.H * L->table.W * L->table.C;
  for (int b = 0; b < L->batch; ++b) {
    if (L->cursor >= L->perm.size()) {
      L->cursor = 0;
      if (L->shuffle) std::shuffle(L->perm.begin(), L->perm.end(), L->rng);
    }
    uint32_t idx = L->perm[L->cursor++];
    std::memcpy(L->img_slots[slot] + b * per, L->table.images.data() + idx * per, per);
    L->lab_slots[slot][b] = L->table.labels[idx];
  }
}

void worker_main(Loader* L) {
  while (!L->stop) {
    int slot;
    {
      std::unique_lock<std::mutex> lk(L->mu);
      L->cv.wait(lk, [&] { return L->stop || L->state[L->next_fill] == 0; });
      if (L->stop) return;
      slot = L->next_fill;
      L->state[slot] = 1;
      L->next_fill = (L->next_fill + 1) % L->nslots;
    }
    fill(L, slot);
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->state[slot] = 2;
    }
    L->cv.notify_all();
  }
}
}  // namespace

// files: '\n'-separated list. label_bytes: 1 (CIFAR-10) or 2 (CIFAR-100)
API void* dtm_cifar_table_open(const char* files, int label_bytes) {
  Loader* L = new Loader();
  std::string all(files);
  size_t s = 0;
  while (s < all.size()) {
    size_t e = all.find('\n', s);
    if (e == std::string::npos) e = all.size();
    std::string p = all.substr(s, e - s);
    if (!p.empty() && !load_cifar_file(p.c_str(), label_bytes, &L->table)) {
      delete L;
      return nullptr;
    }
    s = e + 1;
  }
  return L;
}

API int64_t dtm_cifar_table_size(void* h) { return (int64_t)((Loader*)h)->table.n(); }

// copy records [start, start+n) (no shuffling) -- evaluation path
API int dtm_cifar_table_get(void* h, int64_t start, int n, uint8_t* images, int32_t* labels) {
  Loader* L = (Loader*)h;
  const size_t per = 3072;
  for (int i = 0; i < n; ++i) {
    size_t idx = (size_t)((start + i) % (int64_t)L->table.n());
    std::memcpy(images + i * per, L->table.images.data() + idx * per, per);
    labels[i] = L->table.labels[idx];
  }
  return 0;
}

// start the prefetch ring over caller-owned slots (img: nslots*batch*3072 bytes, lab: nslots*batch int32)
API int dtm_loader_start(void* h, int batch, int nslots, uint8_t* img, int32_t* lab, int shuffle, uint64_t seed) {
  Loader* L = (Loader*)h;
  if (L->table.n() == 0 || nslots < 1) return -1;
  L->batch = batch;
  L->nslots = nslots;
  L->shuffle = shuffle != 0;
  L->rng.seed(seed);
  L->perm.resize(L->table.n());
  for (size_t i = 0; i < L->perm.size(); ++i) L->perm[i] = (uint32_t)i;
  if (L->shuffle) std::shuffle(L->perm.begin(), L->perm.end(), L->rng);
  const size_t per = (size_t)batch * 3072;
  for (int s = 0; s < nslots; ++s) {
    L->img_slots.push_back(img + s * per);
    L->lab_slots.push_back(lab + (size_t)s * batch);
  }
  L->state.assign(nslots, 0);
  L->worker = std::thread(worker_main, L);
  return 0;
}

// block until the next slot is ready; returns its index
API int dtm_loader_next(void* h) {
  Loader* L = (Loader*)h;
  std::unique_lock<std::mutex> lk(L->mu);
  L->cv.wait(lk, [&] { return L->state[L->next_get] == 2; });
  int s = L->next_get;
  L->next_get = (L->next_get + 1) % L->nslots;
  return s;
}

API void dtm_loader_release(void* h, int slot) {
  Loader* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->state[slot] = 0;
  }
  L->cv.notify_all();
}

API void dtm_cifar_table_close(void* h) {
  Loader* L = (Loader*)h;
  if (L->worker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(L->mu);
      L->stop = true;
    }
    L->cv.notify_all();
    L->worker.join();
  }
  delete L;
}
