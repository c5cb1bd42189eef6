// fuzz_dap.cpp -- AddressSanitizer harness for the host side of the DAP codec (SURVEY.md 5:
// "ASan host build"): janus_dap_agg_init_scan / janus_dap_agg_init_unpack_host parse untrusted
// AggregationJobInitializeReq bodies, so they are run here on mutated bodies (bit flips, byte
// sets, truncations, length-field edits, record splices) under -fsanitize=address, with output
// buffers sized exactly as janus_dap.h specifies for the layout the scan returned.
// Build + run: make -C janus_amd asan  (no GPU needed: only host entry points are called).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../include/janus_dap.h"

namespace {

void put_be(std::vector<uint8_t>& b, uint64_t v, int n) {
  for (int i = n - 1; i >= 0; i--) b.push_back((uint8_t)(v >> (8 * i)));
}

// a well-formed body: TimeInterval query, n PrepareInits of random shapes
std::vector<uint8_t> make_body(std::mt19937_64& g, int n) {
  std::vector<uint8_t> recs;
  for (int r = 0; r < n; r++) {
    for (int i = 0; i < 16; i++) recs.push_back((uint8_t)g());
    put_be(recs, 1700000000 + g() % 3600, 8);
    const uint32_t psl = (g() % 4 == 0) ? (uint32_t)(g() % 40) : 32;
    put_be(recs, psl, 4);
    for (uint32_t i = 0; i < psl; i++) recs.push_back((uint8_t)g());
    recs.push_back(7);
    put_be(recs, 32, 2);
    for (int i = 0; i < 32; i++) recs.push_back((uint8_t)g());
    const uint32_t pay = 40 + g() % 40;
    put_be(recs, pay, 4);
    for (uint32_t i = 0; i < pay; i++) recs.push_back((uint8_t)g());
    const uint32_t ty = g() % 8 == 0 ? (uint32_t)(g() % 3) : 0u;
    const uint32_t psl2 = 48;
    std::vector<uint8_t> msg{(uint8_t)ty};
    if (ty == 1) {  // Continue { prep_msg, prep_share }
      put_be(msg, 16, 4);
      for (int i = 0; i < 16; i++) msg.push_back((uint8_t)g());
    }
    put_be(msg, psl2, 4);
    for (uint32_t i = 0; i < psl2; i++) msg.push_back((uint8_t)g());
    put_be(recs, msg.size(), 4);
    recs.insert(recs.end(), msg.begin(), msg.end());
  }
  std::vector<uint8_t> b;
  put_be(b, 0, 4);  // aggregation parameter <u32>
  b.push_back(1);   // query type TimeInterval
  put_be(b, recs.size(), 4);
  b.insert(b.end(), recs.begin(), recs.end());
  return b;
}

void mutate(std::mt19937_64& g, std::vector<uint8_t>& b) {
  const int k = 1 + (int)(g() % 4);
  for (int i = 0; i < k && !b.empty(); i++) {
    const size_t at = g() % b.size();
    switch (g() % 5) {
      case 0: b[at] ^= (uint8_t)(1u << (g() % 8)); break;
      case 1: b[at] = (uint8_t)g(); break;
      case 2: b.resize(at); break;                                     // truncate
      case 3: b[at] = (uint8_t)(g() % 2 ? 0xff : 0x00); break;          // length extremes
      default: {                                                        // splice a chunk
        const size_t from = g() % b.size(), len = std::min<size_t>(g() % 64, b.size() - from);
        std::vector<uint8_t> chunk(b.begin() + from, b.begin() + from + len);
        b.insert(b.begin() + at, chunk.begin(), chunk.end());
      }
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 20000;
  std::mt19937_64 g(argc > 2 ? strtoull(argv[2], nullptr, 10) : 0x4a414e5553ull);
  long scanned = 0, unpacked = 0, rejected = 0;
  for (long it = 0; it < iters; it++) {
    std::vector<uint8_t> body = make_body(g, 1 + (int)(g() % 12));
    if (it % 8) mutate(g, body);
    // exact-size copy: an over-read past the body is an ASan error
    uint8_t* buf = (uint8_t*)malloc(body.size() ? body.size() : 1);
    memcpy(buf, body.data(), body.size());
    janus_dap_agg_init_layout L;
    memset(&L, 0, sizeof L);
    if (janus_dap_agg_init_scan(buf, body.size(), &L) != 0) {
      rejected++;
      free(buf);
      continue;
    }
    scanned++;
    // records are >= 16+8+4+1+2+4+4 = 39 bytes: cap bounds the count of any decodable list
    const uint32_t cap = (uint32_t)(L.list_len / 39 + 1);
    const uint32_t ct_stride = ((L.payload_len + 15) / 16) * 16 + 16;
    std::vector<uint8_t> ids(16 * (size_t)cap), pub((size_t)L.public_share_len * cap + 1),
        cfg(cap), enc((size_t)L.enc_len * cap + 1), ct((size_t)ct_stride * cap),
        ps((size_t)L.prep_share_len * cap + 1), st(cap);
    std::vector<uint64_t> times(cap);
    std::vector<uint32_t> ctl(cap);
    const int64_t n = janus_dap_agg_init_unpack_host(
        buf, body.size(), &L, cap, ids.data(), times.data(), pub.data(), cfg.data(), enc.data(),
        ct.data(), ctl.data(), ct_stride, ps.data(), st.data());
    if (n >= 0) {
      unpacked++;
      for (int64_t r = 0; r < n; r++)
        if (st[r] != 0 && st[r] != 2 && st[r] != 5 && st[r] != 6) {
          fprintf(stderr, "bad msg_status %u\n", st[r]);
          return 1;
        }
    }
    free(buf);
  }
  printf("fuzz_dap: %ld bodies, %ld scanned, %ld unpacked, %ld rejected at scan -- no ASan "
         "report\n", iters, scanned, unpacked, rejected);
  return 0;
}
