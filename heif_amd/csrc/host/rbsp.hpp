// rbsp.hpp — RBSP bit reader and emulation-prevention removal.
// Mirrors src/hevc/rbsp_reader.rs (RbspReader::remove_emulation_prevention
// :11-39, read_bits/read_ue/read_se/byte_alignment :53-136): same rule for
// 00 00 03 xx (xx <= 3 or at end), MSB-first bits, errors on EOF.
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace hg {

struct HeifError : std::runtime_error {
    explicit HeifError(const std::string &m) : std::runtime_error(m) {}
};
// a valid stream that uses a tool outside this decode path (HEIFGPU_E_UNSUPPORTED)
struct UnsupportedError : HeifError {
    explicit UnsupportedError(const std::string &m) : HeifError(m) {}
};

class RbspReader {
  public:
    RbspReader(const uint8_t *data, size_t len) : d_(data), n_(len) {}

    // rbsp_reader.rs:11-39. If ep_raw is non-null it receives the raw index of
    // every removed 0x03 byte (used to map RBSP offsets back to entry points).
    static std::vector<uint8_t> remove_emulation_prevention(const uint8_t *in, size_t n,
                                                            std::vector<uint32_t> *ep_raw = nullptr);

    bool is_byte_aligned() const { return (bit_ & 7) == 0; }
    size_t bit_position() const { return bit_; }
    size_t byte_position() const { return bit_ >> 3; }
    size_t bits_left() const { return n_ * 8 > bit_ ? n_ * 8 - bit_ : 0; }

    uint32_t read_bit() {
        if ((bit_ >> 3) >= n_) throw HeifError("unexpected EOF in RBSP");
        uint32_t b = (d_[bit_ >> 3] >> (7 - (bit_ & 7))) & 1u;
        ++bit_;
        return b;
    }
    bool read_flag() { return read_bit() != 0; }
    uint32_t read_bits(int n) {
        if (n > 32) throw HeifError("read_bits > 32");
        uint32_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 1) | read_bit();
        return v;
    }
    uint32_t read_ue() {
        int lz = 0;
        while (!read_bit())
            if (++lz > 31) throw HeifError("ue(v) too long");
        if (lz == 0) return 0;
        return ((1u << lz) - 1u) + read_bits(lz);
    }
    // ue(v) with its semantic range checked before any narrowing cast
    int read_ue_max(uint32_t max, const char *what) {
        const uint32_t v = read_ue();
        if (v > max) throw HeifError(std::string(what) + " out of range");
        return int(v);
    }
    int32_t read_se() {
        uint32_t k = read_ue();
        if (k == 0) return 0;
        return (k & 1) ? int32_t((k + 1) / 2) : -int32_t(k / 2);
    }
    int read_se_range(int lo, int hi, const char *what) {
        const int32_t v = read_se();
        if (v < lo || v > hi) throw HeifError(std::string(what) + " out of range");
        return v;
    }
    // byte_alignment(): alignment_bit_equal_to_one then zero bits (rbsp_reader.rs:53-63)
    void byte_alignment() {
        if (read_bit() != 1) throw HeifError("byte_alignment: expected 1");
        while (!is_byte_aligned())
            if (read_bit() != 0) throw HeifError("byte_alignment: expected 0");
    }
    void skip_bits(size_t n) { bit_ += n; }

  private:
    const uint8_t *d_;
    size_t n_;
    size_t bit_ = 0;
};

}  // namespace hg
