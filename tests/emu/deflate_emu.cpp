// CPU emulation driver for hsds_amd/csrc/deflate_wave.h (TEST INFRASTRUCTURE ONLY).
// Runs the exact single-source phases of the wave encoder (parse -> Huffman ->
// layout -> emit) with LANE_LOOP iterating the 64 lanes in order, for one zlib
// stream, so that the orchestration is checked against libz inflate on CPU.  Never
// used by the product.
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "../../hsds_amd/csrc/deflate_wave.h"
#include "../../hsds_amd/csrc/lz4_enc.h"
#include "../../hsds_amd/csrc/zstd_enc.h"

// far: the HBM far-chain ring is handed over (the parse uses it when tune.far, as the engine)
static int64_t run(const hd::EncJob& job, const hd::Tune& tune, uint8_t* dst, uint32_t cap, int far = 1) {
  const uint32_t nseg = hd::nsegments(job.len);
  std::vector<hd::SegParse> sp(nseg);
  std::vector<hd::SegCode> sc(nseg);
  std::vector<uint16_t> tok((size_t)nseg * hd::SEG_TOK);
  hd::ParseShared* ps = (hd::ParseShared*)calloc(1, sizeof(hd::ParseShared));
  hd::HuffShared* hs = (hd::HuffShared*)calloc(1, sizeof(hd::HuffShared));
  hd::EmitShared* es = (hd::EmitShared*)calloc(1, sizeof(hd::EmitShared));
  std::vector<uint16_t> fr(hd::FARW, 0);
  const uint32_t adler = hd::parse_stream(*ps, job, tune, sp.data(), tok.data(), nullptr, far ? fr.data() : nullptr);
  for (uint32_t s = 0; s < nseg; s++) {
    const uint32_t s0 = s * (uint32_t)hd::SEG;
    const uint32_t seglen = job.len - s0 < (uint32_t)hd::SEG ? job.len - s0 : (uint32_t)hd::SEG;
    hd::huff_segment(*hs, &sp[s], &sc[s], seglen, tune.stored);
  }
  const uint64_t total = hd::stream_layout(sc.data(), job.len, nullptr);
  int64_t r = -1;
  if (total <= cap) {
    // the layout phase: block bit positions from bit 16, zlib header bytes
    std::vector<uint32_t> words((total + 8) / 4 + 8, 0u);
    uint8_t* wb = (uint8_t*)words.data();
    wb[0] = 0x78;
    wb[1] = (uint8_t)hd::zlib_flg(job.level);
    uint64_t bpos = 16;
    for (uint32_t s = 0; s < nseg; s++) {
      const uint32_t s0 = s * (uint32_t)hd::SEG;
      const uint32_t seglen = job.len - s0 < (uint32_t)hd::SEG ? job.len - s0 : (uint32_t)hd::SEG;
      hd::SegOut o;
      o.bitpos = bpos;
      o.item = 0;
      o.seg = s;
      o.flags = 1u | (s + 1 == nseg ? 2u : 0u);
      o.adler = adler;
      hd::emit_segment(*es, o, &sc[s], &sp[s], tok.data() + (size_t)s * hd::SEG_TOK, job, words.data());
      if (sc[s].btype == 0) bpos = ((bpos + 3u + 7u) & ~7ull) + 32u + 8ull * seglen;
      else bpos += sc[s].bits;
    }
    memcpy(dst, wb, total);
    r = (int64_t)total;
  }
  free(ps);
  free(hs);
  free(es);
  return r;
}

// Returns compressed bytes or -1 when they would exceed cap.
extern "C" int64_t emu_deflate(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level,
                               int chain_override) {
  hd::Tune tune = hd::tune_for_level(level);
  if (chain_override > 0) tune.chain = (uint32_t)chain_override;
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  return run(job, tune, dst, cap);
}

// far = 0 / 1: the parse without / with the far ring at any level (size comparison in the tests)
extern "C" int64_t emu_deflate_far(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level,
                                   int chain_override, int far) {
  hd::Tune tune = hd::tune_for_level(level);
  if (chain_override > 0) tune.chain = (uint32_t)chain_override;
  tune.far = far ? 1u : 0u;
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  return run(job, tune, dst, cap);
}

// gather mode: the stream is bytes [off, off + n) of the byte-shuffled block at src
extern "C" int64_t emu_deflate_shuffled(const uint8_t* block, uint32_t n, uint8_t* dst, uint32_t cap, int level,
                                        uint32_t ts, uint32_t neb, uint32_t off) {
  hd::EncJob job = {block, n, level, ts, neb, off};
  return run(job, hd::tune_for_level(level), dst, cap);
}

// LZ4 block of one split: the parse phase, then the lz4_enc.h token walk (size pass,
// then write pass).  Returns the block size or -1 when it would exceed cap.
extern "C" int64_t emu_lz4_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level) {
  const uint32_t nseg = hd::nsegments(n);
  std::vector<hd::SegParse> sp(nseg);
  std::vector<uint16_t> tok((size_t)nseg * hd::SEG_TOK);
  hd::ParseShared* ps = (hd::ParseShared*)calloc(1, sizeof(hd::ParseShared));
  hd::Tune tune = hd::tune_for_level(level);
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  hd::parse_stream(*ps, job, tune, sp.data(), tok.data());
  free(ps);
  const uint32_t sz = lze::lz4_block_wave(sp.data(), tok.data(), job, nullptr, 0);
  if (sz > cap) return -1;
  lze::CopyList* cl = (lze::CopyList*)calloc(1, sizeof(lze::CopyList));   // the kernel's LDS run list
  const uint32_t sz2 = lze::lz4_block_wave(sp.data(), tok.data(), job, dst, 1, cl);
  free(cl);
  return sz2 == sz ? (int64_t)sz : -2;
}

// BloscLZ block of one split (parse phase, then lz4_enc.h blosclz_block_wave)
extern "C" int64_t emu_blosclz_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level) {
  const uint32_t nseg = hd::nsegments(n);
  std::vector<hd::SegParse> sp(nseg);
  std::vector<uint16_t> tok((size_t)nseg * hd::SEG_TOK);
  hd::ParseShared* ps = (hd::ParseShared*)calloc(1, sizeof(hd::ParseShared));
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  hd::parse_stream(*ps, job, hd::tune_for_level(level), sp.data(), tok.data());
  free(ps);
  const uint32_t sz = lze::blosclz_block_wave(sp.data(), tok.data(), job, nullptr, 0);
  if (sz > cap) return -1;
  const uint32_t sz2 = lze::blosclz_block_wave(sp.data(), tok.data(), job, dst, 1);
  return sz2 == sz ? (int64_t)sz : -2;
}

// zstd frame of one Blosc block (the zstd writer): parse, then one zstd block per 8 KiB
// segment (zstd_enc.h), behind the frame header.  Returns the frame size or -1 past cap.
// tables: 1 = the frame's FSE_Compressed_Mode sequence tables (the engine's), 0 = predefined
extern "C" int64_t emu_zstd_frame_t(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level, int tables);
extern "C" int64_t emu_zstd_frame(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level) {
  return emu_zstd_frame_t(src, n, dst, cap, level, 1);
}
static int g_zstd_seqs = 0;     // 1: the zstd_seq_kernel path (compact sequences, literals pre-written)
extern "C" void emu_zstd_set_seqs(int on) { g_zstd_seqs = on; }
extern "C" int64_t emu_zstd_frame_t(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap, int level, int tables) {
  const uint32_t nseg = hd::nsegments(n);
  std::vector<hd::SegParse> sp(nseg);
  std::vector<uint16_t> tok((size_t)nseg * hd::SEG_TOK);
  hd::ParseShared* ps = (hd::ParseShared*)calloc(1, sizeof(hd::ParseShared));
  std::vector<uint16_t> fr(hd::FARW, 0);
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  hd::parse_stream(*ps, job, hd::tune_for_level(level), sp.data(), tok.data(), nullptr, fr.data());
  free(ps);
  hze::Tabs T;
  hze::build_all(T);
  hze::CodeTabs ct;
  hze::code_tabs_fill(ct, 0u, 1u);
  if (tables) {
    hze::SeqCounts c;
    memset(&c, 0, sizeof(c));
    for (uint32_t s = 0; s < nseg; s++) hze::count_segment(ct, tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], c);
    hze::frame_tables(T, c);
  }
  std::vector<uint8_t> blk(hze::ZCAP), lsec(hze::LCAP);
  hze::LitShared* ls = (hze::LitShared*)calloc(1, sizeof(hze::LitShared));
  uint8_t hdr[16];
  const uint32_t h = hze::frame_header(hdr, n);
  uint64_t pos = 0;
  auto put = [&](const uint8_t* p, uint32_t k) {
    for (uint32_t i = 0; i < k; i++, pos++) if (pos < cap) dst[pos] = p[i];
  };
  put(hdr, h);
  for (uint32_t s = 0; s < nseg; s++) {
    const uint32_t s0 = s * (uint32_t)hd::SEG;
    const uint32_t seglen = n - s0 < (uint32_t)hd::SEG ? n - s0 : (uint32_t)hd::SEG;
    const uint32_t lsz = !hze::huff_lit_level(level) ? 0u
                         : hze::lit_section(*ls, tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], lsec.data());
    if (g_zstd_seqs) {
      std::fill(blk.begin(), blk.end(), (uint8_t)0xA5);
      hze::extract_sequences(tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], blk.data(), lsz == 0u);
    }
    const uint32_t k = hze::encode_segment(T, ct, tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], job, s0, seglen,
                                           s + 1 == nseg ? 1u : 0u, blk.data(), hze::ZCAP, lsec.data(), lsz,
                                           g_zstd_seqs);
    put(blk.data(), k);
  }
  free(ls);
  return pos <= cap ? (int64_t)pos : -1;
}

extern "C" int emu_parse_shared_bytes() { return (int)sizeof(hd::ParseShared); }
extern "C" int emu_huff_shared_bytes() { return (int)sizeof(hd::HuffShared); }
extern "C" int emu_emit_shared_bytes() { return (int)sizeof(hd::EmitShared); }

// the sequence-code counts of a zstd frame's segments two ways: count_segment (the serial
// backward sequence walk encode_segment uses) into c_walk, and zstd_count_kernel's per-lane
// algorithm (count_segment_lanes) into c_lanes; 121 u32 each.  Returns the segment count.
extern "C" int emu_zstd_counts(const uint8_t* src, uint32_t n, int level, uint32_t* c_walk, uint32_t* c_lanes) {
  const uint32_t nseg = hd::nsegments(n);
  std::vector<hd::SegParse> sp(nseg);
  std::vector<uint16_t> tok((size_t)nseg * hd::SEG_TOK);
  hd::ParseShared* ps = (hd::ParseShared*)calloc(1, sizeof(hd::ParseShared));
  std::vector<uint16_t> fr(hd::FARW, 0);
  hd::EncJob job = {src, n, level, 1u, 0u, 0u};
  hd::parse_stream(*ps, job, hd::tune_for_level(level), sp.data(), tok.data(), nullptr, fr.data());
  free(ps);
  hze::CodeTabs ct;
  hze::code_tabs_fill(ct, 0u, 1u);
  hze::SeqCounts a, b;
  memset(&a, 0, sizeof(a));
  memset(&b, 0, sizeof(b));
  for (uint32_t s = 0; s < nseg; s++) {
    hze::count_segment(ct, tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], a);
    hze::count_segment_lanes(ct, tok.data() + (size_t)s * hd::SEG_TOK, &sp[s], b);
  }
  memcpy(c_walk, &a, sizeof(a));
  memcpy(c_lanes, &b, sizeof(b));
  return (int)nseg;
}
