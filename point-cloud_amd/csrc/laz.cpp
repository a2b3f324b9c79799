// laz.cpp — LASzip "pointwise chunked" codec for LAS point formats 0-3 (see laz.h).
//
// Coder and models follow the LASzip 2.x design (Amir Said's FastAC adaptive
// arithmetic coder): 32-bit interval, renormalisation below 2^24, symbol models
// with periodically rebuilt distributions (and a decoder lookup table above 16
// symbols), binary models with 13-bit probabilities.  IntegerCompressor codes
// a prediction residual as its bit length k (one symbol model per context) and
// the value inside the 2^k interval (symbol models for k <= 8, plus raw bits).
// The item compressors predict each field from the previous point:
//   POINT10 v2   changed-field mask, per-return-type intensity, streaming
//                medians of dx / dy per return type, z per return level;
//   GPSTIME11 v2 multiples of the last time difference over four sequences;
//   RGB12 v2     per-byte differences predicted across channels;
//   BYTE v2      per-byte differences (extra bytes).
#include "laz.h"

#include <string.h>

#include <algorithm>
#include <stdexcept>

namespace pcc {
namespace laz {
namespace {

constexpr uint32_t AC_MinLength = 0x01000000u;
constexpr uint32_t AC_MaxLength = 0xFFFFFFFFu;
constexpr uint32_t BM_LengthShift = 13, BM_MaxCount = 1u << BM_LengthShift;
constexpr uint32_t DM_LengthShift = 15, DM_MaxCount = 1u << DM_LengthShift;

inline uint8_t u8_fold(int32_t n) { return (uint8_t)(n < 0 ? n + 256 : (n > 255 ? n - 256 : n)); }
inline uint8_t u8_clamp(int32_t n) { return (uint8_t)(n <= 0 ? 0 : (n >= 255 ? 255 : n)); }

// ------------------------------------------------------------------ models
struct SymbolModel {
    uint32_t symbols, last_symbol;
    bool compress;
    std::vector<uint32_t> distribution, symbol_count, decoder_table;
    uint32_t total_count = 0, update_cycle = 0, symbols_until_update = 0;
    uint32_t table_size = 0, table_shift = 0;
    SymbolModel(uint32_t n, bool enc) : symbols(n), last_symbol(n - 1), compress(enc) {
        if (n < 2 || n > (1u << 11)) throw std::runtime_error("laz: bad symbol model size");
        if (!enc && n > 16) {
            uint32_t table_bits = 3;
            while (n > (1u << (table_bits + 2))) ++table_bits;
            table_size = 1u << table_bits;
            table_shift = DM_LengthShift - table_bits;
            decoder_table.assign(table_size + 2, 0);
        }
        distribution.assign(n, 0);
        symbol_count.assign(n, 0);
        init();
    }
    void init() {
        total_count = 0;
        update_cycle = symbols;
        for (uint32_t k = 0; k < symbols; k++) symbol_count[k] = 1;
        update();
        symbols_until_update = update_cycle = (symbols + 6) >> 1;
    }
    void update() {
        if ((total_count += update_cycle) > DM_MaxCount) {
            total_count = 0;
            for (uint32_t n = 0; n < symbols; n++) total_count += (symbol_count[n] = (symbol_count[n] + 1) >> 1);
        }
        uint32_t sum = 0, s = 0;
        const uint32_t scale = 0x80000000u / total_count;
        if (compress || table_size == 0) {
            for (uint32_t k = 0; k < symbols; k++) {
                distribution[k] = (scale * sum) >> (31 - DM_LengthShift);
                sum += symbol_count[k];
            }
        } else {
            for (uint32_t k = 0; k < symbols; k++) {
                distribution[k] = (scale * sum) >> (31 - DM_LengthShift);
                sum += symbol_count[k];
                const uint32_t w = distribution[k] >> table_shift;
                while (s < w) decoder_table[++s] = k - 1;
            }
            decoder_table[0] = 0;
            while (s <= table_size) decoder_table[++s] = symbols - 1;
        }
        update_cycle = (5 * update_cycle) >> 2;
        const uint32_t max_cycle = (symbols + 6) << 3;
        if (update_cycle > max_cycle) update_cycle = max_cycle;
        symbols_until_update = update_cycle;
    }
};

struct BitModel {
    uint32_t bit_0_count = 1, bit_count = 2, bit_0_prob = 1u << (BM_LengthShift - 1);
    uint32_t update_cycle = 4, bits_until_update = 4;
    void init() { *this = BitModel(); }
    void update() {
        if ((bit_count += update_cycle) > BM_MaxCount) {
            bit_count = (bit_count + 1) >> 1;
            bit_0_count = (bit_0_count + 1) >> 1;
            if (bit_0_count == bit_count) ++bit_count;
        }
        const uint32_t scale = 0x80000000u / bit_count;
        bit_0_prob = (bit_0_count * scale) >> (31 - BM_LengthShift);
        update_cycle = (5 * update_cycle) >> 2;
        if (update_cycle > 64) update_cycle = 64;
        bits_until_update = update_cycle;
    }
};

// ------------------------------------------------------------------ coders
struct Decoder {
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    uint32_t value = 0, length = 0;
    bool overrun = false;
    uint8_t get() {
        if (p < end) return *p++;
        overrun = true;
        return 0;
    }
    void init(const uint8_t* b, const uint8_t* e) {
        p = b;
        end = e;
        overrun = false;
        length = AC_MaxLength;
        value = (uint32_t)get() << 24;
        value |= (uint32_t)get() << 16;
        value |= (uint32_t)get() << 8;
        value |= (uint32_t)get();
    }
    void renorm() {
        do value = (value << 8) | get();
        while ((length <<= 8) < AC_MinLength);
    }
    uint32_t bit(BitModel& m) {
        const uint32_t x = m.bit_0_prob * (length >> BM_LengthShift);
        uint32_t sym;
        if (value < x) {
            length = x;
            ++m.bit_0_count;
            sym = 0;
        } else {
            value -= x;
            length -= x;
            sym = 1;
        }
        if (length < AC_MinLength) renorm();
        if (--m.bits_until_update == 0) m.update();
        return sym;
    }
    uint32_t symbol(SymbolModel& m) {
        uint32_t n, sym, x, y = length;
        if (!m.decoder_table.empty()) {
            const uint32_t dv = value / (length >>= DM_LengthShift);
            const uint32_t t = dv >> m.table_shift;
            sym = m.decoder_table[t];
            n = m.decoder_table[t + 1] + 1;
            while (n > sym + 1) {
                const uint32_t k = (sym + n) >> 1;
                if (m.distribution[k] > dv) n = k;
                else sym = k;
            }
            x = m.distribution[sym] * length;
            if (sym != m.last_symbol) y = m.distribution[sym + 1] * length;
        } else {
            x = sym = 0;
            length >>= DM_LengthShift;
            uint32_t k = (n = m.symbols) >> 1;
            do {
                const uint32_t z = length * m.distribution[k];
                if (z > value) {
                    n = k;
                    y = z;
                } else {
                    sym = k;
                    x = z;
                }
            } while ((k = (sym + n) >> 1) != sym);
        }
        value -= x;
        length = y - x;
        if (length < AC_MinLength) renorm();
        ++m.symbol_count[sym];
        if (--m.symbols_until_update == 0) m.update();
        return sym;
    }
    uint32_t bits(uint32_t b) {
        if (b > 19) {
            const uint32_t lo = short16();
            const uint32_t hi = bits(b - 16);
            return (hi << 16) | lo;
        }
        const uint32_t sym = value / (length >>= b);
        value -= length * sym;
        if (length < AC_MinLength) renorm();
        return sym;
    }
    uint32_t short16() {
        const uint32_t sym = value / (length >>= 16);
        value -= length * sym;
        if (length < AC_MinLength) renorm();
        return sym;
    }
    uint32_t int32() {
        const uint32_t lo = short16();
        const uint32_t hi = short16();
        return (hi << 16) | lo;
    }
};

struct Encoder {
    std::vector<uint8_t>* out = nullptr;
    uint32_t base = 0, length = 0;
    void init(std::vector<uint8_t>* o) {
        out = o;
        base = 0;
        length = AC_MaxLength;
    }
    void carry() {   // propagate a carry into the bytes already written
        size_t i = out->size();
        while (i > 0 && (*out)[i - 1] == 0xFF) (*out)[--i] = 0;
        if (i > 0) ++(*out)[i - 1];
    }
    void renorm() {
        do {
            out->push_back((uint8_t)(base >> 24));
            base <<= 8;
        } while ((length <<= 8) < AC_MinLength);
    }
    void bit(BitModel& m, uint32_t sym) {
        const uint32_t x = m.bit_0_prob * (length >> BM_LengthShift);
        if (sym == 0) {
            length = x;
            ++m.bit_0_count;
        } else {
            const uint32_t b0 = base;
            base += x;
            length -= x;
            if (b0 > base) carry();
        }
        if (length < AC_MinLength) renorm();
        if (--m.bits_until_update == 0) m.update();
    }
    void symbol(SymbolModel& m, uint32_t sym) {
        uint32_t x;
        const uint32_t b0 = base;
        if (sym == m.last_symbol) {
            x = m.distribution[sym] * (length >> DM_LengthShift);
            base += x;
            length -= x;
        } else {
            x = m.distribution[sym] * (length >>= DM_LengthShift);
            base += x;
            length = m.distribution[sym + 1] * length - x;
        }
        if (b0 > base) carry();
        if (length < AC_MinLength) renorm();
        ++m.symbol_count[sym];
        if (--m.symbols_until_update == 0) m.update();
    }
    void bits(uint32_t b, uint32_t sym) {
        if (b > 19) {
            short16(sym & 0xFFFF);
            sym >>= 16;
            b -= 16;
        }
        const uint32_t b0 = base;
        base += sym * (length >>= b);
        if (b0 > base) carry();
        if (length < AC_MinLength) renorm();
    }
    void short16(uint32_t sym) {
        const uint32_t b0 = base;
        base += sym * (length >>= 16);
        if (b0 > base) carry();
        if (length < AC_MinLength) renorm();
    }
    void int32(uint32_t sym) {
        short16(sym & 0xFFFF);
        short16(sym >> 16);
    }
    void done() {
        const uint32_t b0 = base;
        bool another = true;
        if (length > 2 * AC_MinLength) {
            base += AC_MinLength;
            length = AC_MinLength >> 1;
        } else {
            base += AC_MinLength >> 1;
            length = AC_MinLength >> 9;
            another = false;
        }
        if (b0 > base) carry();
        renorm();
        // the decoder reads four bytes ahead: pad so it never runs past the chunk
        out->push_back(0);
        out->push_back(0);
        if (another) out->push_back(0);
    }
};

// ------------------------------------------------------------------ integer compressor
struct IntegerCompressor {
    uint32_t corr_bits, corr_range, bits_high = 8;
    int32_t corr_min, corr_max;
    uint32_t k = 0;
    std::vector<SymbolModel> mbits;
    BitModel corr0;
    std::vector<SymbolModel> corr;   // corr[i - 1]: k = i
    IntegerCompressor(bool enc, uint32_t bits, uint32_t contexts) {
        if (bits && bits < 32) {
            corr_bits = bits;
            corr_range = 1u << bits;
            corr_min = -(int32_t)(corr_range / 2);
            corr_max = corr_min + (int32_t)corr_range - 1;
        } else {
            corr_bits = 32;
            corr_range = 0;
            corr_min = INT32_MIN;
            corr_max = INT32_MAX;
        }
        for (uint32_t c = 0; c < contexts; c++) mbits.emplace_back(corr_bits + 1, enc);
        for (uint32_t i = 1; i <= corr_bits; i++) corr.emplace_back(i <= bits_high ? (1u << i) : (1u << bits_high), enc);
    }
    void init() {
        for (auto& m : mbits) m.init();
        corr0.init();
        for (auto& m : corr) m.init();
    }
    int32_t decompress(Decoder& d, int32_t pred, uint32_t ctx) {
        int32_t c;
        k = d.symbol(mbits[ctx]);
        if (k) {
            if (k < 32) {
                if (k <= bits_high) {
                    c = (int32_t)d.symbol(corr[k - 1]);
                } else {
                    const uint32_t k1 = k - bits_high;
                    c = (int32_t)d.symbol(corr[k - 1]);
                    const int32_t c1 = (int32_t)d.bits(k1);
                    c = (int32_t)(((uint32_t)c << k1) | (uint32_t)c1);
                }
                // back into [-(2^k - 1), -(2^(k-1))] u [2^(k-1), 2^k]
                if (c >= (int32_t)(1u << (k - 1))) c += 1;
                else c = (int32_t)((uint32_t)c - ((1u << k) - 1));
            } else {
                c = corr_min;
            }
        } else {
            c = (int32_t)d.bit(corr0);
        }
        uint32_t real = (uint32_t)pred + (uint32_t)c;
        if (corr_range) {
            if ((int32_t)real < 0) real += corr_range;
            else if (real >= corr_range) real -= corr_range;
        }
        return (int32_t)real;
    }
    void compress(Encoder& e, int32_t pred, int32_t real, uint32_t ctx) {
        int32_t c = (int32_t)((uint32_t)real - (uint32_t)pred);
        if (corr_range) {
            if (c < corr_min) c = (int32_t)((uint32_t)c + corr_range);
            else if (c > corr_max) c = (int32_t)((uint32_t)c - corr_range);
        }
        // the tightest interval [-(2^k - 1), 2^k] that holds c
        uint32_t c1 = c <= 0 ? (uint32_t)0 - (uint32_t)c : (uint32_t)c - 1;
        k = 0;
        while (c1) {
            c1 >>= 1;
            k++;
        }
        e.symbol(mbits[ctx], k);
        if (k) {
            if (k < 32) {
                uint32_t v = c < 0 ? (uint32_t)c + ((1u << k) - 1) : (uint32_t)c - 1;
                if (k <= bits_high) {
                    e.symbol(corr[k - 1], v);
                } else {
                    const uint32_t k1 = k - bits_high;
                    const uint32_t lo = v & ((1u << k1) - 1);
                    e.symbol(corr[k - 1], v >> k1);
                    e.bits(k1, lo);
                }
            }
        } else {
            e.bit(corr0, (uint32_t)c);
        }
    }
};

// ------------------------------------------------------------------ item codecs
struct Median5 {
    int32_t v[5] = {0, 0, 0, 0, 0};
    bool high = true;
    void init() { *this = Median5(); }
    int32_t get() const { return v[2]; }
    void add(int32_t x) {
        if (high) {
            if (x < v[2]) {
                v[4] = v[3];
                v[3] = v[2];
                if (x < v[0]) { v[2] = v[1]; v[1] = v[0]; v[0] = x; }
                else if (x < v[1]) { v[2] = v[1]; v[1] = x; }
                else v[2] = x;
            } else {
                if (x < v[3]) { v[4] = v[3]; v[3] = x; }
                else v[4] = x;
                high = false;
            }
        } else {
            if (v[2] < x) {
                v[0] = v[1];
                v[1] = v[2];
                if (v[4] < x) { v[2] = v[3]; v[3] = v[4]; v[4] = x; }
                else if (v[3] < x) { v[2] = v[3]; v[3] = x; }
                else v[2] = x;
            } else {
                if (v[1] < x) { v[0] = v[1]; v[1] = x; }
                else v[0] = x;
                high = true;
            }
        }
    }
};

const uint8_t kNumberReturnMap[8][8] = {
    {15, 14, 13, 12, 11, 10, 9, 8},  {14, 0, 1, 3, 6, 10, 10, 9},    {13, 1, 2, 4, 7, 11, 11, 10},
    {12, 3, 4, 5, 8, 12, 12, 11},    {11, 6, 7, 8, 9, 13, 13, 12},   {10, 10, 11, 12, 13, 14, 14, 13},
    {9, 10, 11, 12, 13, 14, 15, 14}, {8, 9, 10, 11, 12, 13, 14, 15}};
const uint8_t kNumberReturnLevel[8][8] = {
    {0, 1, 2, 3, 4, 5, 6, 7}, {1, 0, 1, 2, 3, 4, 5, 6}, {2, 1, 0, 1, 2, 3, 4, 5}, {3, 2, 1, 0, 1, 2, 3, 4},
    {4, 3, 2, 1, 0, 1, 2, 3}, {5, 4, 3, 2, 1, 0, 1, 2}, {6, 5, 4, 3, 2, 1, 0, 1}, {7, 6, 5, 4, 3, 2, 1, 0}};

struct ItemCodec {
    virtual ~ItemCodec() = default;
    virtual void init(const uint8_t* item) = 0;   // first point of a chunk (stored raw)
    virtual void read(Decoder& d, uint8_t* item) = 0;
    virtual void write(Encoder& e, const uint8_t* item) = 0;
};

inline int32_t rd_i32(const uint8_t* p) { int32_t v; memcpy(&v, p, 4); return v; }
inline void wr_i32(uint8_t* p, int32_t v) { memcpy(p, &v, 4); }
inline uint16_t rd_u16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline void wr_u16(uint8_t* p, uint16_t v) { memcpy(p, &v, 2); }

// LASpoint10: x, y, z (i32), intensity (u16), return byte (return number 3 bits,
// number of returns 3, scan direction 1, edge of flight line 1), classification,
// scan angle rank (i8), user data, point source id (u16): 20 bytes
struct Point10 : ItemCodec {
    bool enc;
    uint8_t last[20];
    uint16_t last_intensity[16];
    Median5 mx[16], my[16];
    int32_t last_height[8];
    SymbolModel m_changed;
    std::unique_ptr<SymbolModel> m_bit_byte[256], m_classification[256], m_user_data[256];
    SymbolModel m_scan_angle[2];
    IntegerCompressor ic_intensity, ic_psid, ic_dx, ic_dy, ic_z;
    explicit Point10(bool e)
        : enc(e), m_changed(64, e), m_scan_angle{SymbolModel(256, e), SymbolModel(256, e)}, ic_intensity(e, 16, 4),
          ic_psid(e, 16, 1), ic_dx(e, 32, 2), ic_dy(e, 32, 22), ic_z(e, 32, 20) {}
    SymbolModel& lazy(std::unique_ptr<SymbolModel>* tab, uint8_t i) {
        if (!tab[i]) tab[i].reset(new SymbolModel(256, enc));
        return *tab[i];
    }
    void init(const uint8_t* item) override {
        for (int i = 0; i < 16; i++) {
            mx[i].init();
            my[i].init();
            last_intensity[i] = 0;
            last_height[i / 2] = 0;
        }
        m_changed.init();
        ic_intensity.init();
        m_scan_angle[0].init();
        m_scan_angle[1].init();
        ic_psid.init();
        for (int i = 0; i < 256; i++) {
            if (m_bit_byte[i]) m_bit_byte[i]->init();
            if (m_classification[i]) m_classification[i]->init();
            if (m_user_data[i]) m_user_data[i]->init();
        }
        ic_dx.init();
        ic_dy.init();
        ic_z.init();
        memcpy(last, item, 20);
        last[12] = last[13] = 0;   // the intensity is predicted from zero
    }
    static uint32_t kctx(uint32_t k, uint32_t cap) { return k < cap ? (k & ~1u) : cap; }
    void read(Decoder& d, uint8_t* item) override {
        const uint32_t changed = d.symbol(m_changed);
        uint32_t r, n;
        if (changed) {
            if (changed & 32) last[14] = (uint8_t)d.symbol(lazy(m_bit_byte, last[14]));
            r = last[14] & 7;
            n = (last[14] >> 3) & 7;
            const uint32_t m = kNumberReturnMap[n][r];
            if (changed & 16) {
                const uint16_t it = (uint16_t)ic_intensity.decompress(d, last_intensity[m], m < 3 ? m : 3);
                wr_u16(last + 12, it);
                last_intensity[m] = it;
            } else {
                wr_u16(last + 12, last_intensity[m]);
            }
            if (changed & 8) last[15] = (uint8_t)d.symbol(lazy(m_classification, last[15]));
            if (changed & 4) {
                const int32_t v = (int32_t)d.symbol(m_scan_angle[(last[14] >> 6) & 1]);
                last[16] = u8_fold(v + last[16]);
            }
            if (changed & 2) last[17] = (uint8_t)d.symbol(lazy(m_user_data, last[17]));
            if (changed & 1) wr_u16(last + 18, (uint16_t)ic_psid.decompress(d, rd_u16(last + 18), 0));
        } else {
            r = last[14] & 7;
            n = (last[14] >> 3) & 7;
        }
        const uint32_t m = kNumberReturnMap[n][r], l = kNumberReturnLevel[n][r];
        if (!changed) wr_u16(last + 12, last_intensity[m]);
        int32_t med = mx[m].get();
        int32_t diff = ic_dx.decompress(d, med, n == 1);
        wr_i32(last, (int32_t)((uint32_t)rd_i32(last) + (uint32_t)diff));
        mx[m].add(diff);
        med = my[m].get();
        uint32_t kb = ic_dx.k;
        diff = ic_dy.decompress(d, med, (n == 1) + kctx(kb, 20));
        wr_i32(last + 4, (int32_t)((uint32_t)rd_i32(last + 4) + (uint32_t)diff));
        my[m].add(diff);
        kb = (ic_dx.k + ic_dy.k) / 2;
        const int32_t z = ic_z.decompress(d, last_height[l], (n == 1) + kctx(kb, 18));
        wr_i32(last + 8, z);
        last_height[l] = z;
        memcpy(item, last, 20);
    }
    void write(Encoder& e, const uint8_t* item) override {
        const uint32_t r = item[14] & 7, n = (item[14] >> 3) & 7;
        const uint32_t m = kNumberReturnMap[n][r], l = kNumberReturnLevel[n][r];
        const uint32_t changed = ((last[14] != item[14]) << 5) | ((last_intensity[m] != rd_u16(item + 12)) << 4) |
                                 ((last[15] != item[15]) << 3) | ((last[16] != item[16]) << 2) |
                                 ((last[17] != item[17]) << 1) | (rd_u16(last + 18) != rd_u16(item + 18));
        e.symbol(m_changed, changed);
        if (changed & 32) e.symbol(lazy(m_bit_byte, last[14]), item[14]);
        if (changed & 16) {
            ic_intensity.compress(e, last_intensity[m], rd_u16(item + 12), m < 3 ? m : 3);
            last_intensity[m] = rd_u16(item + 12);
        }
        if (changed & 8) e.symbol(lazy(m_classification, last[15]), item[15]);
        if (changed & 4) e.symbol(m_scan_angle[(item[14] >> 6) & 1], u8_fold((int32_t)item[16] - (int32_t)last[16]));
        if (changed & 2) e.symbol(lazy(m_user_data, last[17]), item[17]);
        if (changed & 1) ic_psid.compress(e, rd_u16(last + 18), rd_u16(item + 18), 0);
        int32_t diff = (int32_t)((uint32_t)rd_i32(item) - (uint32_t)rd_i32(last));
        ic_dx.compress(e, mx[m].get(), diff, n == 1);
        mx[m].add(diff);
        uint32_t kb = ic_dx.k;
        diff = (int32_t)((uint32_t)rd_i32(item + 4) - (uint32_t)rd_i32(last + 4));
        ic_dy.compress(e, my[m].get(), diff, (n == 1) + kctx(kb, 20));
        my[m].add(diff);
        kb = (ic_dx.k + ic_dy.k) / 2;
        ic_z.compress(e, last_height[l], rd_i32(item + 8), (n == 1) + kctx(kb, 18));
        last_height[l] = rd_i32(item + 8);
        memcpy(last, item, 20);
    }
};

constexpr int32_t kGpsMulti = 500, kGpsMultiMinus = -10;
constexpr uint32_t kGpsUnchanged = kGpsMulti - kGpsMultiMinus + 1;   // 511
constexpr uint32_t kGpsCodeFull = kGpsMulti - kGpsMultiMinus + 2;    // 512
constexpr uint32_t kGpsTotal = kGpsMulti - kGpsMultiMinus + 6;       // 516

struct Gps11 : ItemCodec {
    SymbolModel m_multi, m_0diff;
    IntegerCompressor ic;
    uint32_t last = 0, next = 0;
    int64_t gps[4] = {0, 0, 0, 0};
    int32_t diff[4] = {0, 0, 0, 0};
    int32_t extreme[4] = {0, 0, 0, 0};
    explicit Gps11(bool e) : m_multi(kGpsTotal, e), m_0diff(6, e), ic(e, 32, 9) {}
    void init(const uint8_t* item) override {
        last = next = 0;
        for (int i = 0; i < 4; i++) { diff[i] = 0; extreme[i] = 0; gps[i] = 0; }
        m_multi.init();
        m_0diff.init();
        ic.init();
        memcpy(&gps[0], item, 8);
    }
    void full(Decoder& d) {
        next = (next + 1) & 3;
        const uint64_t hi = (uint32_t)ic.decompress(d, (int32_t)((uint64_t)gps[last] >> 32), 8);
        gps[next] = (int64_t)((hi << 32) | d.int32());
        last = next;
        diff[last] = 0;
        extreme[last] = 0;
    }
    void read(Decoder& d, uint8_t* item) override {
        for (;;) {
            if (diff[last] == 0) {
                const uint32_t multi = d.symbol(m_0diff);
                if (multi == 1) {
                    diff[last] = ic.decompress(d, 0, 0);
                    gps[last] = (int64_t)((uint64_t)gps[last] + (uint64_t)(int64_t)diff[last]);
                    extreme[last] = 0;
                } else if (multi == 2) {
                    full(d);
                } else if (multi > 2) {
                    last = (last + multi - 2) & 3;
                    continue;
                }
            } else {
                uint32_t multi = d.symbol(m_multi);
                if (multi == 1) {
                    gps[last] = (int64_t)((uint64_t)gps[last] + (uint64_t)(int64_t)ic.decompress(d, diff[last], 1));
                    extreme[last] = 0;
                } else if (multi < kGpsUnchanged) {
                    int32_t g;
                    if (multi == 0) {
                        g = ic.decompress(d, 0, 7);
                        if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                    } else if (multi < (uint32_t)kGpsMulti) {
                        g = ic.decompress(d, (int32_t)((uint32_t)multi * (uint32_t)diff[last]), multi < 10 ? 2 : 3);
                    } else if (multi == (uint32_t)kGpsMulti) {
                        g = ic.decompress(d, (int32_t)((uint32_t)kGpsMulti * (uint32_t)diff[last]), 4);
                        if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                    } else {
                        const int32_t mm = kGpsMulti - (int32_t)multi;
                        if (mm > kGpsMultiMinus) {
                            g = ic.decompress(d, (int32_t)((uint32_t)mm * (uint32_t)diff[last]), 5);
                        } else {
                            g = ic.decompress(d, (int32_t)((uint32_t)kGpsMultiMinus * (uint32_t)diff[last]), 6);
                            if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                        }
                    }
                    gps[last] = (int64_t)((uint64_t)gps[last] + (uint64_t)(int64_t)g);
                } else if (multi == kGpsCodeFull) {
                    full(d);
                } else if (multi > kGpsCodeFull) {
                    last = (last + multi - kGpsCodeFull) & 3;
                    continue;
                }
            }
            break;
        }
        memcpy(item, &gps[last], 8);
    }
    // Encoder: one sequence (no switching between the four), multiples chosen as
    // LASzip's writer does for a single sequence; enough for the decoder tests.
    void write(Encoder& e, const uint8_t* item) override {
        int64_t t;
        memcpy(&t, item, 8);
        const int64_t dd = (int64_t)((uint64_t)t - (uint64_t)gps[last]);
        const bool fits = dd >= INT32_MIN && dd <= INT32_MAX;
        if (diff[last] == 0) {
            if (dd == 0) {
                e.symbol(m_0diff, 0);
            } else if (fits) {
                e.symbol(m_0diff, 1);
                ic.compress(e, 0, (int32_t)dd, 0);
                diff[last] = (int32_t)dd;
                extreme[last] = 0;
                gps[last] = t;
            } else {
                e.symbol(m_0diff, 2);
                wfull(e, t);
            }
        } else {
            if (dd == 0) {
                e.symbol(m_multi, kGpsUnchanged);
            } else if (fits) {
                const int32_t g = (int32_t)dd;
                // multiple of the last difference, rounded (LASzip's writer)
                const double mf = (double)g / (double)diff[last];
                const int32_t multi = mf > 1e6 ? 1000000 : mf < -1e6 ? -1000000 : (int32_t)(mf >= 0 ? mf + 0.5 : mf - 0.5);
                if (multi == 1) {
                    e.symbol(m_multi, 1);
                    ic.compress(e, diff[last], g, 1);
                    extreme[last] = 0;
                } else if (multi > 0 && multi < kGpsMulti) {
                    e.symbol(m_multi, (uint32_t)multi);
                    ic.compress(e, (int32_t)((uint32_t)multi * (uint32_t)diff[last]), g, multi < 10 ? 2 : 3);
                } else if (multi >= kGpsMulti) {
                    e.symbol(m_multi, kGpsMulti);
                    ic.compress(e, (int32_t)((uint32_t)kGpsMulti * (uint32_t)diff[last]), g, 4);
                    if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                } else if (multi < 0 && multi > kGpsMultiMinus) {
                    e.symbol(m_multi, (uint32_t)(kGpsMulti - multi));
                    ic.compress(e, (int32_t)((uint32_t)multi * (uint32_t)diff[last]), g, 5);
                } else if (multi < 0) {
                    e.symbol(m_multi, (uint32_t)(kGpsMulti - kGpsMultiMinus));
                    ic.compress(e, (int32_t)((uint32_t)kGpsMultiMinus * (uint32_t)diff[last]), g, 6);
                    if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                } else {   // multi == 0
                    e.symbol(m_multi, 0);
                    ic.compress(e, 0, g, 7);
                    if (++extreme[last] > 3) { diff[last] = g; extreme[last] = 0; }
                }
                gps[last] = t;
            } else {
                e.symbol(m_multi, kGpsCodeFull);
                wfull(e, t);
            }
        }
    }
    void wfull(Encoder& e, int64_t t) {
        next = (next + 1) & 3;
        ic.compress(e, (int32_t)((uint64_t)gps[last] >> 32), (int32_t)((uint64_t)t >> 32), 8);
        e.int32((uint32_t)(uint64_t)t);
        last = next;
        gps[last] = t;
        diff[last] = 0;
        extreme[last] = 0;
    }
};

// RGB12 v2 colour model (also RGB14 v3's): which bytes changed, low/high byte
// differences predicted from the red channel's change
void rgb_decode(Decoder& d, SymbolModel& used, std::vector<SymbolModel>& md, const uint16_t* last, uint16_t* c) {
    const uint32_t sym = d.symbol(used);
    if (sym & 1) c[0] = (uint16_t)u8_fold((int32_t)d.symbol(md[0]) + (last[0] & 255));
    else c[0] = last[0] & 0xFF;
    if (sym & 2) c[0] |= (uint16_t)(u8_fold((int32_t)d.symbol(md[1]) + (last[0] >> 8)) << 8);
    else c[0] |= last[0] & 0xFF00;
    if (sym & 64) {
        int32_t diff = (c[0] & 0xFF) - (last[0] & 0xFF);
        if (sym & 4) c[1] = (uint16_t)u8_fold((int32_t)d.symbol(md[2]) + u8_clamp(diff + (last[1] & 255)));
        else c[1] = last[1] & 0xFF;
        if (sym & 16) {
            diff = (diff + ((c[1] & 0xFF) - (last[1] & 0xFF))) / 2;
            c[2] = (uint16_t)u8_fold((int32_t)d.symbol(md[4]) + u8_clamp(diff + (last[2] & 255)));
        } else {
            c[2] = last[2] & 0xFF;
        }
        diff = (c[0] >> 8) - (last[0] >> 8);
        if (sym & 8) c[1] |= (uint16_t)(u8_fold((int32_t)d.symbol(md[3]) + u8_clamp(diff + (last[1] >> 8))) << 8);
        else c[1] |= last[1] & 0xFF00;
        if (sym & 32) {
            diff = (diff + ((c[1] >> 8) - (last[1] >> 8))) / 2;
            c[2] |= (uint16_t)(u8_fold((int32_t)d.symbol(md[5]) + u8_clamp(diff + (last[2] >> 8))) << 8);
        } else {
            c[2] |= last[2] & 0xFF00;
        }
    } else {
        c[1] = c[0];
        c[2] = c[0];
    }
}
uint32_t rgb_encode(Encoder& e, SymbolModel& used, std::vector<SymbolModel>& md, const uint16_t* last, const uint16_t* c) {
    const uint32_t sym = ((last[0] & 0x00FF) != (c[0] & 0x00FF)) | (((last[0] & 0xFF00) != (c[0] & 0xFF00)) << 1) |
                         (((last[1] & 0x00FF) != (c[1] & 0x00FF)) << 2) | (((last[1] & 0xFF00) != (c[1] & 0xFF00)) << 3) |
                         (((last[2] & 0x00FF) != (c[2] & 0x00FF)) << 4) | (((last[2] & 0xFF00) != (c[2] & 0xFF00)) << 5) |
                         (((c[0] & 0x00FF) != (c[1] & 0x00FF) || (c[0] & 0x00FF) != (c[2] & 0x00FF) ||
                           (c[0] & 0xFF00) != (c[1] & 0xFF00) || (c[0] & 0xFF00) != (c[2] & 0xFF00)) << 6);
    e.symbol(used, sym);
    if (sym & 1) e.symbol(md[0], u8_fold((c[0] & 255) - (last[0] & 255)));
    if (sym & 2) e.symbol(md[1], u8_fold((c[0] >> 8) - (last[0] >> 8)));
    if (sym & 64) {
        int32_t diff = (c[0] & 0xFF) - (last[0] & 0xFF);
        if (sym & 4) e.symbol(md[2], u8_fold((c[1] & 255) - u8_clamp(diff + (last[1] & 255))));
        if (sym & 16) {
            diff = (diff + ((c[1] & 0xFF) - (last[1] & 0xFF))) / 2;
            e.symbol(md[4], u8_fold((c[2] & 255) - u8_clamp(diff + (last[2] & 255))));
        }
        diff = (c[0] >> 8) - (last[0] >> 8);
        if (sym & 8) e.symbol(md[3], u8_fold((c[1] >> 8) - u8_clamp(diff + (last[1] >> 8))));
        if (sym & 32) {
            diff = (diff + ((c[1] >> 8) - (last[1] >> 8))) / 2;
            e.symbol(md[5], u8_fold((c[2] >> 8) - u8_clamp(diff + (last[2] >> 8))));
        }
    }
    return sym;
}

struct Rgb12 : ItemCodec {
    SymbolModel m_used;
    std::vector<SymbolModel> m_diff;
    uint16_t last[3] = {0, 0, 0};
    explicit Rgb12(bool e) : m_used(128, e) {
        for (int i = 0; i < 6; i++) m_diff.emplace_back(256, e);
    }
    void init(const uint8_t* item) override {
        m_used.init();
        for (auto& m : m_diff) m.init();
        memcpy(last, item, 6);
    }
    void read(Decoder& d, uint8_t* item) override {
        uint16_t c[3];
        rgb_decode(d, m_used, m_diff, last, c);
        memcpy(last, c, 6);
        memcpy(item, c, 6);
    }
    void write(Encoder& e, const uint8_t* item) override {
        uint16_t c[3];
        memcpy(c, item, 6);
        rgb_encode(e, m_used, m_diff, last, c);
        memcpy(last, c, 6);
    }
};

struct Bytes : ItemCodec {
    uint32_t n;
    std::vector<SymbolModel> m;
    std::vector<uint8_t> last;
    Bytes(bool e, uint32_t count) : n(count), last(count) {
        for (uint32_t i = 0; i < count; i++) m.emplace_back(256, e);
    }
    void init(const uint8_t* item) override {
        for (auto& x : m) x.init();
        memcpy(last.data(), item, n);
    }
    void read(Decoder& d, uint8_t* item) override {
        for (uint32_t i = 0; i < n; i++) {
            item[i] = u8_fold((int32_t)last[i] + (int32_t)d.symbol(m[i]));
            last[i] = item[i];
        }
    }
    void write(Encoder& e, const uint8_t* item) override {
        for (uint32_t i = 0; i < n; i++) {
            e.symbol(m[i], u8_fold((int32_t)item[i] - (int32_t)last[i]));
            last[i] = item[i];
        }
    }
};

// LASwavepacket13 (29 bytes): descriptor index (u8), then byte offset to the
// waveform data (u64), packet size (u32), return point location and x(t),
// y(t), z(t) (f32, coded as their bit patterns).  WAVEPACKET13 v1, the only
// version LASzip has (point formats 4 / 5 of pointwise-chunked files): the
// index as a symbol; the offset as "same", "previous offset + previous size",
// a 32-bit difference (integer compressor, predicted from the last such
// difference) or a raw 64-bit value, the choice coded with a model selected by
// the previous choice; every other field by an integer compressor from the
// previous point (x, y, z sharing one with three contexts).
struct Wave {
    uint64_t offset;
    uint32_t size;
    int32_t ret, x, y, z;
};
inline Wave wave_unpack(const uint8_t* p) {   // the 28 bytes after the index
    Wave w;
    memcpy(&w.offset, p, 8);
    memcpy(&w.size, p + 8, 4);
    memcpy(&w.ret, p + 12, 4);
    memcpy(&w.x, p + 16, 4);
    memcpy(&w.y, p + 20, 4);
    memcpy(&w.z, p + 24, 4);
    return w;
}
inline void wave_pack(const Wave& w, uint8_t* p) {
    memcpy(p, &w.offset, 8);
    memcpy(p + 8, &w.size, 4);
    memcpy(p + 12, &w.ret, 4);
    memcpy(p + 16, &w.x, 4);
    memcpy(p + 20, &w.y, 4);
    memcpy(p + 24, &w.z, 4);
}
struct WaveModels {
    SymbolModel m_index;
    std::vector<SymbolModel> m_offset;   // by the previous offset code
    IntegerCompressor ic_offset, ic_size, ic_ret, ic_xyz;
    int32_t last_diff = 0;
    uint32_t last_sym = 0;
    uint8_t last[29];
    WaveModels(bool e, const uint8_t* item)
        : m_index(256, e), ic_offset(e, 32, 1), ic_size(e, 32, 1), ic_ret(e, 32, 1), ic_xyz(e, 32, 3) {
        for (int i = 0; i < 4; i++) m_offset.emplace_back(4, e);
        init(item);
    }
    void init(const uint8_t* item) {
        m_index.init();
        for (auto& m : m_offset) m.init();
        ic_offset.init();
        ic_size.init();
        ic_ret.init();
        ic_xyz.init();
        last_diff = 0;
        last_sym = 0;
        memcpy(last, item, 29);
    }
    void read(Decoder& d, uint8_t* item) {
        item[0] = (uint8_t)d.symbol(m_index);
        const Wave lw = wave_unpack(last + 1);
        Wave w;
        last_sym = d.symbol(m_offset[last_sym]);
        if (last_sym == 0) {
            w.offset = lw.offset;
        } else if (last_sym == 1) {
            w.offset = lw.offset + lw.size;
        } else if (last_sym == 2) {
            last_diff = ic_offset.decompress(d, last_diff, 0);
            w.offset = lw.offset + (uint64_t)(int64_t)last_diff;
        } else {
            const uint64_t lo = d.int32();
            const uint64_t hi = d.int32();
            w.offset = (hi << 32) | lo;
        }
        w.size = (uint32_t)ic_size.decompress(d, (int32_t)lw.size, 0);
        w.ret = ic_ret.decompress(d, lw.ret, 0);
        w.x = ic_xyz.decompress(d, lw.x, 0);
        w.y = ic_xyz.decompress(d, lw.y, 1);
        w.z = ic_xyz.decompress(d, lw.z, 2);
        wave_pack(w, item + 1);
        memcpy(last, item, 29);
    }
    void write(Encoder& e, const uint8_t* item) {
        e.symbol(m_index, item[0]);
        const Wave lw = wave_unpack(last + 1), w = wave_unpack(item + 1);
        const int64_t d64 = (int64_t)(w.offset - lw.offset);
        const int32_t d32 = (int32_t)d64;
        uint32_t sym;
        if (d64 == (int64_t)d32) sym = d32 == 0 ? 0u : (d32 == (int32_t)lw.size ? 1u : 2u);
        else sym = 3;
        e.symbol(m_offset[last_sym], sym);
        last_sym = sym;
        if (sym == 2) {
            ic_offset.compress(e, last_diff, d32, 0);
            last_diff = d32;
        } else if (sym == 3) {
            e.int32((uint32_t)w.offset);
            e.int32((uint32_t)(w.offset >> 32));
        }
        ic_size.compress(e, (int32_t)lw.size, (int32_t)w.size, 0);
        ic_ret.compress(e, lw.ret, w.ret, 0);
        ic_xyz.compress(e, lw.x, w.x, 0);
        ic_xyz.compress(e, lw.y, w.y, 1);
        ic_xyz.compress(e, lw.z, w.z, 2);
        memcpy(last, item, 29);
    }
};

struct Wave13 : ItemCodec {
    WaveModels M;
    explicit Wave13(bool e) : M(e, kZero29) {}
    static constexpr uint8_t kZero29[29] = {};
    void init(const uint8_t* item) override { M.init(item); }
    void read(Decoder& d, uint8_t* item) override { M.read(d, item); }
    void write(Encoder& e, const uint8_t* item) override { M.write(e, item); }
};

// ------------------------------------------------------------------ LASzip 3 layered items
// Point formats 6-8 (LAS 1.4): POINT14 v3, RGB14 v3, RGBNIR14 v3, BYTE14 v3 in
// "layered chunked" compression.  Every field group is its own arithmetic
// stream (layer) per chunk, and a layer whose values never change in a chunk
// is stored empty (the decoder then keeps the chunk's first value).  Models
// live in one of four contexts, selected by the point's scanner channel; a
// context is created, from the previous context's last point, when its
// channel first appears in the chunk.
struct LayeredItem {
    virtual ~LayeredItem() = default;
    virtual uint32_t layers() const = 0;
    // decoder: the chunk's first point (stored raw) and this item's layers
    virtual void init_dec(const uint8_t* item, uint32_t& ctx, const uint8_t* const* lp, const uint32_t* ln) = 0;
    virtual void read(uint8_t* item, uint32_t& ctx) = 0;
    virtual bool overrun() const = 0;
    // encoder
    virtual void init_enc(const uint8_t* item, uint32_t& ctx) = 0;
    virtual void write(const uint8_t* item, uint32_t& ctx) = 0;
    virtual void finish(std::vector<std::vector<uint8_t>>& out) = 0;   // layers() streams, empty if unchanged
};

struct LayerSet {   // a layered item's streams
    std::vector<Decoder> dec;
    std::vector<bool> present, changed;
    std::vector<Encoder> enc;
    std::vector<std::vector<uint8_t>> buf;
    explicit LayerSet(uint32_t n) : dec(n), present(n, false), changed(n, false), enc(n), buf(n) {}
    void init_dec(const uint8_t* const* lp, const uint32_t* ln) {
        for (size_t i = 0; i < dec.size(); i++) {
            present[i] = ln[i] > 0;
            if (present[i]) dec[i].init(lp[i], lp[i] + ln[i]);
        }
    }
    void init_enc() {
        for (size_t i = 0; i < enc.size(); i++) {
            buf[i].clear();
            enc[i].init(&buf[i]);
            changed[i] = false;
        }
    }
    void finish(std::vector<std::vector<uint8_t>>& out, bool always_first) {
        for (size_t i = 0; i < enc.size(); i++) {
            enc[i].done();
            out.push_back((changed[i] || (always_first && i == 0)) ? buf[i] : std::vector<uint8_t>());
        }
    }
    bool overrun() const {
        for (const Decoder& d : dec)
            if (d.overrun) return true;
        return false;
    }
};

inline std::unique_ptr<SymbolModel>& lazy_init(std::unique_ptr<SymbolModel>& m, uint32_t n, bool enc) {
    if (!m) m.reset(new SymbolModel(n, enc));
    return m;
}

// The 30-byte LAS 1.4 point record: x, y, z (i32), intensity (u16), returns
// byte (return number bits 0-3, number of returns 4-7), flags byte
// (classification flags 0-3, scanner channel 4-5, scan direction 6, edge of
// flight line 7), classification, user data, scan angle (i16), point source
// id (u16), GPS time (f64)
struct P14 {
    int32_t x = 0, y = 0, z = 0;
    uint16_t intensity = 0, psid = 0;
    uint8_t r = 0, n = 0, cflags = 0, channel = 0, dir = 0, edge = 0, cls = 0, user = 0;
    int16_t angle = 0;
    int64_t gps = 0;
    bool gps_change = false;
};
P14 unpack14(const uint8_t* p) {
    P14 q;
    q.x = rd_i32(p);
    q.y = rd_i32(p + 4);
    q.z = rd_i32(p + 8);
    q.intensity = rd_u16(p + 12);
    q.r = p[14] & 15;
    q.n = p[14] >> 4;
    q.cflags = p[15] & 15;
    q.channel = (p[15] >> 4) & 3;
    q.dir = (p[15] >> 6) & 1;
    q.edge = p[15] >> 7;
    q.cls = p[16];
    q.user = p[17];
    q.angle = (int16_t)rd_u16(p + 18);
    q.psid = rd_u16(p + 20);
    memcpy(&q.gps, p + 22, 8);
    return q;
}
void pack14(const P14& q, uint8_t* p) {
    wr_i32(p, q.x);
    wr_i32(p + 4, q.y);
    wr_i32(p + 8, q.z);
    wr_u16(p + 12, q.intensity);
    p[14] = (uint8_t)(q.r | (q.n << 4));
    p[15] = (uint8_t)(q.cflags | (q.channel << 4) | (q.dir << 6) | (q.edge << 7));
    p[16] = q.cls;
    p[17] = q.user;
    wr_u16(p + 18, (uint16_t)q.angle);
    wr_u16(p + 20, q.psid);
    memcpy(p + 22, &q.gps, 8);
}

// return-type context (6) and return level (8) of (number of returns, return number)
const uint8_t kReturnMap6[16][16] = {
    {0, 1, 2, 3, 4, 5, 3, 4, 4, 5, 5, 5, 5, 5, 5, 5}, {1, 0, 1, 3, 4, 5, 3, 4, 4, 5, 5, 5, 5, 5, 5, 5},
    {2, 1, 2, 4, 4, 5, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5}, {3, 3, 4, 5, 4, 5, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5},
    {4, 4, 4, 4, 5, 5, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5}, {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5},
    {3, 3, 4, 4, 4, 5, 5, 4, 4, 5, 5, 5, 5, 5, 5, 5}, {4, 4, 4, 4, 4, 5, 4, 5, 4, 5, 5, 5, 5, 5, 5, 5},
    {4, 4, 4, 4, 4, 5, 4, 4, 5, 5, 5, 5, 5, 5, 5, 5}, {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5},
    {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5}, {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5},
    {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5}, {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5},
    {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5}, {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5}};
inline uint32_t return_level8(uint32_t n, uint32_t r) { return std::min<uint32_t>(n > r ? n - r : r - n, 7); }

// GPS time codes of the layered coder: no "unchanged" code (the layer is only
// coded for points whose time changed)
constexpr uint32_t kGps3CodeFull = kGpsMulti - kGpsMultiMinus + 1;   // 511
constexpr uint32_t kGps3Total = kGpsMulti - kGpsMultiMinus + 5;      // 515

struct P14Ctx {
    P14 last;
    std::vector<SymbolModel> m_changed;
    SymbolModel m_scanner, m_rn_same, m_gps_multi, m_gps_0diff;
    std::unique_ptr<SymbolModel> m_nret[16], m_rnum[16], m_class[64], m_flags[64], m_user[64];
    IntegerCompressor ic_dx, ic_dy, ic_z, ic_int, ic_angle, ic_psid, ic_gps;
    Median5 mx[12], my[12];
    int32_t last_z[8];
    uint16_t last_int[8];
    uint32_t glast = 0, gnext = 0;
    int64_t gps[4] = {0, 0, 0, 0};
    int32_t gdiff[4] = {0, 0, 0, 0}, gext[4] = {0, 0, 0, 0};
    P14Ctx(bool e, const P14& item)
        : last(item), m_scanner(3, e), m_rn_same(13, e), m_gps_multi(kGps3Total, e), m_gps_0diff(5, e),
          ic_dx(e, 32, 2), ic_dy(e, 32, 22), ic_z(e, 32, 20), ic_int(e, 16, 4), ic_angle(e, 16, 2), ic_psid(e, 16, 1),
          ic_gps(e, 32, 9) {
        for (int i = 0; i < 8; i++) m_changed.emplace_back(128, e);
        for (IntegerCompressor* ic : {&ic_dx, &ic_dy, &ic_z, &ic_int, &ic_angle, &ic_psid, &ic_gps}) ic->init();
        for (int i = 0; i < 8; i++) {
            last_z[i] = item.z;
            last_int[i] = item.intensity;
        }
        last.gps_change = false;
        gps[0] = item.gps;
    }
};

// LASzip 3 POINT14 (layer order: channel/returns/XY, Z, classification, flags,
// intensity, scan angle, user data, point source, GPS time)
struct Point14 : LayeredItem {
    bool enc;
    std::unique_ptr<P14Ctx> C[4];
    uint32_t cur = 0;
    LayerSet L{9};
    explicit Point14(bool e) : enc(e) {}
    uint32_t layers() const override { return 9; }
    bool overrun() const override { return L.overrun(); }
    void start(const uint8_t* item, uint32_t& ctx) {
        const P14 p = unpack14(item);
        for (auto& c : C) c.reset();
        cur = p.channel;
        ctx = cur;
        C[cur].reset(new P14Ctx(enc, p));
    }
    void init_dec(const uint8_t* item, uint32_t& ctx, const uint8_t* const* lp, const uint32_t* ln) override {
        start(item, ctx);
        L.init_dec(lp, ln);
    }
    void init_enc(const uint8_t* item, uint32_t& ctx) override {
        start(item, ctx);
        L.init_enc();
    }
    void finish(std::vector<std::vector<uint8_t>>& out) override { L.finish(out, true); }
    static uint32_t kctx(uint32_t k, uint32_t cap) { return k < cap ? (k & ~1u) : cap; }

    void gps_full(P14Ctx& c, Decoder& d) {
        c.gnext = (c.gnext + 1) & 3;
        const uint64_t hi = (uint32_t)c.ic_gps.decompress(d, (int32_t)((uint64_t)c.gps[c.glast] >> 32), 8);
        c.gps[c.gnext] = (int64_t)((hi << 32) | d.int32());
        c.glast = c.gnext;
        c.gdiff[c.glast] = 0;
        c.gext[c.glast] = 0;
    }
    void read_gps(P14Ctx& c, Decoder& d) {
        for (;;) {
            uint32_t& l = c.glast;
            if (c.gdiff[l] == 0) {
                const uint32_t multi = d.symbol(c.m_gps_0diff);
                if (multi == 0) {
                    c.gdiff[l] = c.ic_gps.decompress(d, 0, 0);
                    c.gps[l] = (int64_t)((uint64_t)c.gps[l] + (uint64_t)(int64_t)c.gdiff[l]);
                    c.gext[l] = 0;
                } else if (multi == 1) {
                    gps_full(c, d);
                } else {
                    l = (l + multi - 1) & 3;
                    continue;
                }
            } else {
                const uint32_t multi = d.symbol(c.m_gps_multi);
                if (multi == 1) {
                    c.gps[l] = (int64_t)((uint64_t)c.gps[l] + (uint64_t)(int64_t)c.ic_gps.decompress(d, c.gdiff[l], 1));
                    c.gext[l] = 0;
                } else if (multi < kGps3CodeFull) {
                    int32_t g;
                    if (multi == 0) {
                        g = c.ic_gps.decompress(d, 0, 7);
                        if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
                    } else if (multi < (uint32_t)kGpsMulti) {
                        g = c.ic_gps.decompress(d, (int32_t)(multi * (uint32_t)c.gdiff[l]), multi < 10 ? 2 : 3);
                    } else if (multi == (uint32_t)kGpsMulti) {
                        g = c.ic_gps.decompress(d, (int32_t)((uint32_t)kGpsMulti * (uint32_t)c.gdiff[l]), 4);
                        if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
                    } else {
                        const int32_t mm = kGpsMulti - (int32_t)multi;
                        if (mm > kGpsMultiMinus) {
                            g = c.ic_gps.decompress(d, (int32_t)((uint32_t)mm * (uint32_t)c.gdiff[l]), 5);
                        } else {
                            g = c.ic_gps.decompress(d, (int32_t)((uint32_t)kGpsMultiMinus * (uint32_t)c.gdiff[l]), 6);
                            if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
                        }
                    }
                    c.gps[l] = (int64_t)((uint64_t)c.gps[l] + (uint64_t)(int64_t)g);
                } else if (multi == kGps3CodeFull) {
                    gps_full(c, d);
                } else {
                    l = (l + multi - kGps3CodeFull) & 3;
                    continue;
                }
            }
            break;
        }
    }
    // encoder: one time sequence per context (the decoder's four-sequence
    // switching is never needed to reproduce the input)
    void write_gps(P14Ctx& c, Encoder& e, int64_t t) {
        uint32_t& l = c.glast;
        const int64_t dd = (int64_t)((uint64_t)t - (uint64_t)c.gps[l]);
        const bool fits = dd >= INT32_MIN && dd <= INT32_MAX;
        auto full = [&]() {
            c.gnext = (c.gnext + 1) & 3;
            c.ic_gps.compress(e, (int32_t)((uint64_t)c.gps[l] >> 32), (int32_t)((uint64_t)t >> 32), 8);
            e.int32((uint32_t)(uint64_t)t);
            l = c.gnext;
            c.gps[l] = t;
            c.gdiff[l] = 0;
            c.gext[l] = 0;
        };
        if (c.gdiff[l] == 0) {
            if (fits) {
                e.symbol(c.m_gps_0diff, 0);
                c.ic_gps.compress(e, 0, (int32_t)dd, 0);
                c.gdiff[l] = (int32_t)dd;
                c.gext[l] = 0;
                c.gps[l] = t;
            } else {
                e.symbol(c.m_gps_0diff, 1);
                full();
            }
            return;
        }
        if (!fits) {
            e.symbol(c.m_gps_multi, kGps3CodeFull);
            full();
            return;
        }
        const int32_t g = (int32_t)dd, df = c.gdiff[l];
        const double mf = (double)g / (double)df;
        const int32_t multi = mf > 1e6 ? 1000000 : mf < -1e6 ? -1000000 : (int32_t)(mf >= 0 ? mf + 0.5 : mf - 0.5);
        if (multi == 1) {
            e.symbol(c.m_gps_multi, 1);
            c.ic_gps.compress(e, df, g, 1);
            c.gext[l] = 0;
        } else if (multi > 0 && multi < kGpsMulti) {
            e.symbol(c.m_gps_multi, (uint32_t)multi);
            c.ic_gps.compress(e, (int32_t)((uint32_t)multi * (uint32_t)df), g, multi < 10 ? 2 : 3);
        } else if (multi >= kGpsMulti) {
            e.symbol(c.m_gps_multi, kGpsMulti);
            c.ic_gps.compress(e, (int32_t)((uint32_t)kGpsMulti * (uint32_t)df), g, 4);
            if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
        } else if (multi < 0 && multi > kGpsMultiMinus) {
            e.symbol(c.m_gps_multi, (uint32_t)(kGpsMulti - multi));
            c.ic_gps.compress(e, (int32_t)((uint32_t)multi * (uint32_t)df), g, 5);
        } else if (multi < 0) {
            e.symbol(c.m_gps_multi, (uint32_t)(kGpsMulti - kGpsMultiMinus));
            c.ic_gps.compress(e, (int32_t)((uint32_t)kGpsMultiMinus * (uint32_t)df), g, 6);
            if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
        } else {
            e.symbol(c.m_gps_multi, 0);
            c.ic_gps.compress(e, 0, g, 7);
            if (++c.gext[l] > 3) { c.gdiff[l] = g; c.gext[l] = 0; }
        }
        c.gps[l] = t;
    }

    void read(uint8_t* item, uint32_t& ctx) override {
        P14Ctx* c = C[cur].get();
        P14* q = &c->last;
        Decoder& d0 = L.dec[0];
        const uint32_t lpr = (q->r == 1 ? 1u : 0u) + (q->r >= q->n ? 2u : 0u) + (q->gps_change ? 4u : 0u);
        const uint32_t changed = d0.symbol(c->m_changed[lpr]);
        if (changed & 64) {   // scanner channel: next = current + diff + 1 (mod 4)
            const uint32_t nc = (cur + d0.symbol(c->m_scanner) + 1) & 3;
            if (!C[nc]) C[nc].reset(new P14Ctx(false, *q));
            cur = nc;
            c = C[cur].get();
            q = &c->last;
            q->channel = (uint8_t)nc;
        }
        ctx = cur;
        const bool psc = (changed & 32) != 0, gpsc = (changed & 16) != 0, angc = (changed & 8) != 0;
        const uint32_t last_n = q->n, last_r = q->r;
        const uint32_t n = (changed & 4) ? d0.symbol(*lazy_init(c->m_nret[last_n], 16, false)) : last_n;
        uint32_t r;
        switch (changed & 3) {
            case 0: r = last_r; break;
            case 1: r = (last_r + 1) & 15; break;
            case 2: r = (last_r + 15) & 15; break;
            default:
                r = gpsc ? d0.symbol(*lazy_init(c->m_rnum[last_r], 16, false))
                         : (last_r + d0.symbol(c->m_rn_same) + 2) & 15;
        }
        q->n = (uint8_t)n;
        q->r = (uint8_t)r;
        const uint32_t m = kReturnMap6[n][r], lv = return_level8(n, r);
        const uint32_t cpr = (r == 1 ? 2u : 0u) + (r >= n ? 1u : 0u);
        const uint32_t mi = (m << 1) | (gpsc ? 1u : 0u);
        int32_t diff = c->ic_dx.decompress(d0, c->mx[mi].get(), n == 1);
        q->x = (int32_t)((uint32_t)q->x + (uint32_t)diff);
        c->mx[mi].add(diff);
        diff = c->ic_dy.decompress(d0, c->my[mi].get(), (n == 1) + kctx(c->ic_dx.k, 20));
        q->y = (int32_t)((uint32_t)q->y + (uint32_t)diff);
        c->my[mi].add(diff);
        if (L.present[1]) {
            const uint32_t kb = (c->ic_dx.k + c->ic_dy.k) / 2;
            q->z = c->ic_z.decompress(L.dec[1], c->last_z[lv], (n == 1) + kctx(kb, 18));
            c->last_z[lv] = q->z;
        }
        if (L.present[2]) {
            const uint32_t ccc = ((q->cls & 0x1Fu) << 1) + (cpr == 3 ? 1u : 0u);
            q->cls = (uint8_t)L.dec[2].symbol(*lazy_init(c->m_class[ccc], 256, false));
        }
        if (L.present[3]) {
            const uint32_t lf = (q->edge << 5) | (q->dir << 4) | q->cflags;
            const uint32_t f = L.dec[3].symbol(*lazy_init(c->m_flags[lf], 64, false));
            q->edge = (f >> 5) & 1;
            q->dir = (f >> 4) & 1;
            q->cflags = f & 15;
        }
        if (L.present[4]) {
            const uint32_t li = (cpr << 1) | (gpsc ? 1u : 0u);
            q->intensity = (uint16_t)c->ic_int.decompress(L.dec[4], c->last_int[li], cpr);
            c->last_int[li] = q->intensity;
        }
        if (L.present[5] && angc) q->angle = (int16_t)c->ic_angle.decompress(L.dec[5], q->angle, gpsc ? 1 : 0);
        if (L.present[6]) q->user = (uint8_t)L.dec[6].symbol(*lazy_init(c->m_user[q->user / 4], 256, false));
        if (L.present[7] && psc) q->psid = (uint16_t)c->ic_psid.decompress(L.dec[7], q->psid, 0);
        if (L.present[8] && gpsc) {
            read_gps(*c, L.dec[8]);
            q->gps = c->gps[c->glast];
        }
        pack14(*q, item);
        q->gps_change = gpsc;
    }

    void write(const uint8_t* item, uint32_t& ctx) override {
        const P14 p = unpack14(item);
        P14Ctx* c = C[cur].get();
        const P14& q0 = c->last;
        const uint32_t lpr = (q0.r == 1 ? 1u : 0u) + (q0.r >= q0.n ? 2u : 0u) + (q0.gps_change ? 4u : 0u);
        const bool sw = p.channel != cur;
        P14Ctx* nc = c;
        if (sw) {
            if (!C[p.channel]) C[p.channel].reset(new P14Ctx(true, q0));
            nc = C[p.channel].get();
        }
        P14& q = nc->last;
        const bool psc = p.psid != q.psid, gpsc = p.gps != q.gps, angc = p.angle != q.angle;
        uint32_t rcode = 3;
        if (p.r == q.r) rcode = 0;
        else if (p.r == ((q.r + 1) & 15)) rcode = 1;
        else if (p.r == ((q.r + 15) & 15)) rcode = 2;
        const uint32_t changed = (sw ? 64u : 0u) | (psc ? 32u : 0u) | (gpsc ? 16u : 0u) | (angc ? 8u : 0u) |
                                 (p.n != q.n ? 4u : 0u) | rcode;
        Encoder& e0 = L.enc[0];
        e0.symbol(c->m_changed[lpr], changed);
        if (sw) {
            e0.symbol(c->m_scanner, (p.channel + 4 - cur - 1) & 3);
            cur = p.channel;
            q.channel = p.channel;
            c = nc;
        }
        ctx = cur;
        if (p.n != q.n) e0.symbol(*lazy_init(c->m_nret[q.n], 16, true), p.n);
        if (rcode == 3) {
            if (gpsc) e0.symbol(*lazy_init(c->m_rnum[q.r], 16, true), p.r);
            else e0.symbol(c->m_rn_same, (p.r + 16 - q.r - 2) & 15);
        }
        const uint32_t n = p.n, r = p.r;
        const uint32_t m = kReturnMap6[n][r], lv = return_level8(n, r);
        const uint32_t cpr = (r == 1 ? 2u : 0u) + (r >= n ? 1u : 0u);
        const uint32_t mi = (m << 1) | (gpsc ? 1u : 0u);
        int32_t diff = (int32_t)((uint32_t)p.x - (uint32_t)q.x);
        c->ic_dx.compress(e0, c->mx[mi].get(), diff, n == 1);
        c->mx[mi].add(diff);
        diff = (int32_t)((uint32_t)p.y - (uint32_t)q.y);
        c->ic_dy.compress(e0, c->my[mi].get(), diff, (n == 1) + kctx(c->ic_dx.k, 20));
        c->my[mi].add(diff);
        const uint32_t kb = (c->ic_dx.k + c->ic_dy.k) / 2;
        c->ic_z.compress(L.enc[1], c->last_z[lv], p.z, (n == 1) + kctx(kb, 18));
        c->last_z[lv] = p.z;
        L.changed[1] = L.changed[1] || p.z != q.z;
        const uint32_t ccc = ((q.cls & 0x1Fu) << 1) + (cpr == 3 ? 1u : 0u);
        L.enc[2].symbol(*lazy_init(c->m_class[ccc], 256, true), p.cls);
        L.changed[2] = L.changed[2] || p.cls != q.cls;
        const uint32_t lf = (q.edge << 5) | (q.dir << 4) | q.cflags, f = (p.edge << 5) | (p.dir << 4) | p.cflags;
        L.enc[3].symbol(*lazy_init(c->m_flags[lf], 64, true), f);
        L.changed[3] = L.changed[3] || f != lf;
        const uint32_t li = (cpr << 1) | (gpsc ? 1u : 0u);
        c->ic_int.compress(L.enc[4], c->last_int[li], p.intensity, cpr);
        c->last_int[li] = p.intensity;
        L.changed[4] = L.changed[4] || p.intensity != q.intensity;
        if (angc) {
            c->ic_angle.compress(L.enc[5], q.angle, p.angle, gpsc ? 1 : 0);
            L.changed[5] = true;
        }
        L.enc[6].symbol(*lazy_init(c->m_user[q.user / 4], 256, true), p.user);
        L.changed[6] = L.changed[6] || p.user != q.user;
        if (psc) {
            c->ic_psid.compress(L.enc[7], q.psid, p.psid, 0);
            L.changed[7] = true;
        }
        if (gpsc) {
            write_gps(*c, L.enc[8], p.gps);
            L.changed[8] = true;
        }
        q = p;
        q.gps_change = gpsc;
    }
};

// RGB14 v3 (colour layer) and RGBNIR14 v3 (plus a near-infrared layer): the
// RGB12 v2 model per context
struct RgbCtx {
    SymbolModel m_used;
    std::vector<SymbolModel> m_diff;
    SymbolModel m_nir_used;
    std::vector<SymbolModel> m_nir;
    uint16_t last[4];
    RgbCtx(bool e, const uint16_t* item) : m_used(128, e), m_nir_used(4, e) {
        for (int i = 0; i < 6; i++) m_diff.emplace_back(256, e);
        for (int i = 0; i < 2; i++) m_nir.emplace_back(256, e);
        memcpy(last, item, 8);
    }
};

struct Rgb14 : LayeredItem {
    bool enc, nir;
    std::unique_ptr<RgbCtx> C[4];
    uint32_t cur = 0;
    LayerSet L;
    Rgb14(bool e, bool with_nir) : enc(e), nir(with_nir), L(with_nir ? 2 : 1) {}
    uint32_t layers() const override { return nir ? 2 : 1; }
    bool overrun() const override { return L.overrun(); }
    void start(const uint8_t* item, uint32_t ctx) {
        uint16_t v[4] = {0, 0, 0, 0};
        memcpy(v, item, nir ? 8 : 6);
        for (auto& c : C) c.reset();
        cur = ctx;
        C[cur].reset(new RgbCtx(enc, v));
    }
    void init_dec(const uint8_t* item, uint32_t& ctx, const uint8_t* const* lp, const uint32_t* ln) override {
        start(item, ctx);
        L.init_dec(lp, ln);
    }
    void init_enc(const uint8_t* item, uint32_t& ctx) override {
        start(item, ctx);
        L.init_enc();
    }
    void finish(std::vector<std::vector<uint8_t>>& out) override { L.finish(out, false); }
    RgbCtx* switch_to(uint32_t ctx) {
        if (ctx != cur) {
            if (!C[ctx]) C[ctx].reset(new RgbCtx(enc, C[cur]->last));
            cur = ctx;
        }
        return C[cur].get();
    }
    void read(uint8_t* item, uint32_t& ctx) override {
        RgbCtx* c = switch_to(ctx);
        uint16_t v[4];
        memcpy(v, c->last, 8);
        if (L.present[0]) rgb_decode(L.dec[0], c->m_used, c->m_diff, c->last, v);
        if (nir && L.present[1]) {
            Decoder& d = L.dec[1];
            const uint32_t sym = d.symbol(c->m_nir_used);
            uint16_t w = (sym & 1) ? u8_fold((int32_t)d.symbol(c->m_nir[0]) + (c->last[3] & 255)) : (c->last[3] & 0xFF);
            w |= (sym & 2) ? (uint16_t)(u8_fold((int32_t)d.symbol(c->m_nir[1]) + (c->last[3] >> 8)) << 8)
                           : (uint16_t)(c->last[3] & 0xFF00);
            v[3] = w;
        }
        memcpy(c->last, v, 8);
        memcpy(item, v, nir ? 8 : 6);
    }
    void write(const uint8_t* item, uint32_t& ctx) override {
        RgbCtx* c = switch_to(ctx);
        uint16_t v[4] = {0, 0, 0, 0};
        memcpy(v, item, nir ? 8 : 6);
        if (rgb_encode(L.enc[0], c->m_used, c->m_diff, c->last, v)) L.changed[0] = true;
        if (nir) {
            const uint32_t sym = ((c->last[3] & 0xFF) != (v[3] & 0xFF)) | (((c->last[3] & 0xFF00) != (v[3] & 0xFF00)) << 1);
            Encoder& e = L.enc[1];
            e.symbol(c->m_nir_used, sym);
            if (sym & 1) e.symbol(c->m_nir[0], u8_fold((v[3] & 255) - (c->last[3] & 255)));
            if (sym & 2) e.symbol(c->m_nir[1], u8_fold((v[3] >> 8) - (c->last[3] >> 8)));
            if (sym) L.changed[1] = true;
        }
        memcpy(c->last, v, 8);
    }
};

// BYTE14 v3: one layer per extra byte, per-byte differences
struct Bytes14 : LayeredItem {
    bool enc;
    uint32_t nb;
    struct Ctx {
        std::vector<SymbolModel> m;
        std::vector<uint8_t> last;
    };
    std::unique_ptr<Ctx> C[4];
    uint32_t cur = 0;
    LayerSet L;
    Bytes14(bool e, uint32_t n) : enc(e), nb(n), L(n) {}
    uint32_t layers() const override { return nb; }
    bool overrun() const override { return L.overrun(); }
    Ctx* make(const uint8_t* item) {
        Ctx* c = new Ctx();
        for (uint32_t i = 0; i < nb; i++) c->m.emplace_back(256, enc);
        c->last.assign(item, item + nb);
        return c;
    }
    void start(const uint8_t* item, uint32_t ctx) {
        for (auto& c : C) c.reset();
        cur = ctx;
        C[cur].reset(make(item));
    }
    void init_dec(const uint8_t* item, uint32_t& ctx, const uint8_t* const* lp, const uint32_t* ln) override {
        start(item, ctx);
        L.init_dec(lp, ln);
    }
    void init_enc(const uint8_t* item, uint32_t& ctx) override {
        start(item, ctx);
        L.init_enc();
    }
    void finish(std::vector<std::vector<uint8_t>>& out) override { L.finish(out, false); }
    Ctx* switch_to(uint32_t ctx) {
        if (ctx != cur) {
            if (!C[ctx]) C[ctx].reset(make(C[cur]->last.data()));
            cur = ctx;
        }
        return C[cur].get();
    }
    void read(uint8_t* item, uint32_t& ctx) override {
        Ctx* c = switch_to(ctx);
        for (uint32_t i = 0; i < nb; i++) {
            if (L.present[i]) c->last[i] = u8_fold((int32_t)c->last[i] + (int32_t)L.dec[i].symbol(c->m[i]));
            item[i] = c->last[i];
        }
    }
    void write(const uint8_t* item, uint32_t& ctx) override {
        Ctx* c = switch_to(ctx);
        for (uint32_t i = 0; i < nb; i++) {
            const int32_t diff = (int32_t)item[i] - (int32_t)c->last[i];
            L.enc[i].symbol(c->m[i], u8_fold(diff));
            if (diff) L.changed[i] = true;
            c->last[i] = item[i];
        }
    }
};

// WAVEPACKET14 v3 (point formats 9 / 10): one layer, the WAVEPACKET13 model
// per scanner-channel context (a new context starts from the previous
// context's last packet); an empty layer keeps the chunk's first packet.
struct Wave14 : LayeredItem {
    bool enc;
    std::unique_ptr<WaveModels> C[4];
    uint32_t cur = 0;
    LayerSet L;
    explicit Wave14(bool e) : enc(e), L(1) {}
    uint32_t layers() const override { return 1; }
    bool overrun() const override { return L.overrun(); }
    void start(const uint8_t* item, uint32_t ctx) {
        for (auto& c : C) c.reset();
        cur = ctx;
        C[cur].reset(new WaveModels(enc, item));
    }
    void init_dec(const uint8_t* item, uint32_t& ctx, const uint8_t* const* lp, const uint32_t* ln) override {
        start(item, ctx);
        L.init_dec(lp, ln);
    }
    void init_enc(const uint8_t* item, uint32_t& ctx) override {
        start(item, ctx);
        L.init_enc();
    }
    void finish(std::vector<std::vector<uint8_t>>& out) override { L.finish(out, false); }
    WaveModels* switch_to(uint32_t ctx) {
        if (ctx != cur) {
            if (!C[ctx]) C[ctx].reset(new WaveModels(enc, C[cur]->last));
            cur = ctx;
        }
        return C[cur].get();
    }
    void read(uint8_t* item, uint32_t& ctx) override {
        WaveModels* c = switch_to(ctx);
        if (L.present[0]) c->read(L.dec[0], item);
        else memcpy(item, c->last, 29);
    }
    void write(const uint8_t* item, uint32_t& ctx) override {
        WaveModels* c = switch_to(ctx);
        if (memcmp(item, c->last, 29) != 0) L.changed[0] = true;
        c->write(L.enc[0], item);
    }
};

bool is_layered(const std::vector<Item>& items) { return !items.empty() && items[0].type == POINT14; }

bool make_layered(const std::vector<Item>& items, bool enc, std::vector<std::unique_ptr<LayeredItem>>& out,
                  std::string& err) {
    out.clear();
    for (size_t i = 0; i < items.size(); i++) {
        const Item& it = items[i];
        if (it.version != 3) {
            err = "LAZ item type " + std::to_string(it.type) + " version " + std::to_string(it.version) + " is not supported";
            return false;
        }
        if (i == 0 ? (it.type == POINT14 && it.size == 30) : false) out.emplace_back(new Point14(enc));
        else if (i > 0 && it.type == RGB14 && it.size == 6) out.emplace_back(new Rgb14(enc, false));
        else if (i > 0 && it.type == RGBNIR14 && it.size == 8) out.emplace_back(new Rgb14(enc, true));
        else if (i > 0 && it.type == BYTE14 && it.size >= 1) out.emplace_back(new Bytes14(enc, it.size));
        else if (i > 0 && it.type == WAVEPACKET14 && it.size == 29) out.emplace_back(new Wave14(enc));
        else {
            err = "LAZ item type " + std::to_string(it.type) + " (size " + std::to_string(it.size) +
                  ") is not supported in layered compression";
            return false;
        }
    }
    return true;
}

bool make_codecs(const std::vector<Item>& items, bool enc, std::vector<std::unique_ptr<ItemCodec>>& out,
                 std::string& err) {
    out.clear();
    for (const Item& it : items) {
        if (it.type == POINT10 && it.size == 20 && it.version == 2) out.emplace_back(new Point10(enc));
        else if (it.type == GPSTIME11 && it.size == 8 && it.version == 2) out.emplace_back(new Gps11(enc));
        else if (it.type == RGB12 && it.size == 6 && it.version == 2) out.emplace_back(new Rgb12(enc));
        else if (it.type == BYTE && it.size >= 1 && it.version == 2) out.emplace_back(new Bytes(enc, it.size));
        else if (it.type == WAVEPACKET13 && it.size == 29 && it.version == 1) out.emplace_back(new Wave13(enc));
        else {
            err = "LAZ item type " + std::to_string(it.type) + " version " + std::to_string(it.version) +
                  (it.type >= POINT14 ? " (point formats 6-10, layered compression)" : "") + " is not supported";
            return false;
        }
    }
    return true;
}

}  // namespace

// ------------------------------------------------------------------ point decoder
class PointDecoder {
public:
    std::vector<std::unique_ptr<ItemCodec>> codecs;
    std::vector<std::unique_ptr<LayeredItem>> layered;   // compressor 3
    std::vector<uint16_t> sizes;
    Decoder dec;
    bool first = true;
    uint32_t ctx = 0;
};

bool parse_vlr(const uint8_t* d, size_t n, Vlr& v, std::string& err) {
    if (n < 34) { err = "LASzip VLR too short"; return false; }
    auto u16 = [&](size_t o) { uint16_t x; memcpy(&x, d + o, 2); return x; };
    auto u32 = [&](size_t o) { uint32_t x; memcpy(&x, d + o, 4); return x; };
    auto i64 = [&](size_t o) { int64_t x; memcpy(&x, d + o, 8); return x; };
    v.compressor = u16(0);
    v.coder = u16(2);
    v.version_major = d[4];
    v.version_minor = d[5];
    v.version_revision = u16(6);
    v.options = u32(8);
    v.chunk_size = u32(12);
    v.number_of_special_evlrs = i64(16);
    v.offset_to_special_evlrs = i64(24);
    const uint16_t ni = u16(32);
    if (n < 34 + 6ull * ni) { err = "LASzip VLR too short for its items"; return false; }
    v.items.clear();
    for (uint16_t i = 0; i < ni; i++) v.items.push_back({u16(34 + 6 * i), u16(36 + 6 * i), u16(38 + 6 * i)});
    return true;
}

std::vector<uint8_t> write_vlr(const Vlr& v) {
    std::vector<uint8_t> d(34 + 6 * v.items.size());
    auto p16 = [&](size_t o, uint16_t x) { memcpy(d.data() + o, &x, 2); };
    auto p32 = [&](size_t o, uint32_t x) { memcpy(d.data() + o, &x, 4); };
    auto p64 = [&](size_t o, int64_t x) { memcpy(d.data() + o, &x, 8); };
    p16(0, v.compressor);
    p16(2, v.coder);
    d[4] = v.version_major;
    d[5] = v.version_minor;
    p16(6, v.version_revision);
    p32(8, v.options);
    p32(12, v.chunk_size);
    p64(16, v.number_of_special_evlrs);
    p64(24, v.offset_to_special_evlrs);
    p16(32, (uint16_t)v.items.size());
    for (size_t i = 0; i < v.items.size(); i++) {
        p16(34 + 6 * i, v.items[i].type);
        p16(36 + 6 * i, v.items[i].size);
        p16(38 + 6 * i, v.items[i].version);
    }
    return d;
}

uint16_t compressor_for_format(uint8_t format) { return format >= 6 ? 3 : 2; }

bool items_for_format(uint8_t format, uint16_t rec, std::vector<Item>& items, std::string& err) {
    static const uint16_t base[11] = {20, 28, 26, 34, 57, 63, 30, 36, 38, 59, 67};
    if (format > 10) {
        err = "LAZ point format " + std::to_string(format) + " is not supported";
        return false;
    }
    if (rec < base[format]) { err = "point record shorter than its format"; return false; }
    items.clear();
    if (format >= 6) {
        items.push_back({POINT14, 30, 3});
        if (format == 7) items.push_back({RGB14, 6, 3});
        if (format == 8 || format == 10) items.push_back({RGBNIR14, 8, 3});
        if (format >= 9) items.push_back({WAVEPACKET14, 29, 3});
        if (rec > base[format]) items.push_back({BYTE14, (uint16_t)(rec - base[format]), 3});
        return true;
    }
    items.push_back({POINT10, 20, 2});
    if (format == 1 || format == 3 || format == 4 || format == 5) items.push_back({GPSTIME11, 8, 2});
    if (format == 2 || format == 3 || format == 5) items.push_back({RGB12, 6, 2});
    if (format == 4 || format == 5) items.push_back({WAVEPACKET13, 29, 1});   // LASzip has no version 2
    if (rec > base[format]) items.push_back({BYTE, (uint16_t)(rec - base[format]), 2});
    return true;
}

Reader::Reader() = default;
Reader::~Reader() = default;

bool Reader::open(FILE* f, uint64_t data_off, uint64_t npoints, uint16_t rec, const Vlr& v, std::string& err) {
    f_ = f;
    rec_ = rec;
    left_ = npoints;
    v_ = v;
    if (v.coder != 0) { err = "LAZ coder " + std::to_string(v.coder) + " is not supported"; return false; }
    const bool layered = is_layered(v.items);
    if (layered ? v.compressor != 3 : (v.compressor != 1 && v.compressor != 2)) {
        err = "LAZ compressor " + std::to_string(v.compressor) + " does not match its items";
        return false;
    }
    uint32_t sum = 0;
    for (const Item& it : v.items) sum += it.size;
    if (sum != rec) { err = "LAZ items do not add up to the point record length"; return false; }
    dec_.reset(new PointDecoder());
    if (layered ? !make_layered(v.items, false, dec_->layered, err) : !make_codecs(v.items, false, dec_->codecs, err))
        return false;
    for (const Item& it : v.items) dec_->sizes.push_back(it.size);
    chunk_start_.clear();
    chunk_pts_.clear();
    if (fseeko(f, (off_t)data_off, SEEK_SET) != 0) { err = "bad offset to point data"; return false; }
    if (fseeko(f, 0, SEEK_END) != 0) { err = "cannot seek"; return false; }
    const uint64_t fsize = (uint64_t)ftello(f);
    if (v.compressor == 1) {   // one stream from the point data to the end of the file
        chunk_start_ = {data_off, fsize};
        chunk_pts_ = {npoints};
    } else {
        int64_t table = -1;
        fseeko(f, (off_t)data_off, SEEK_SET);
        if (fread(&table, 8, 1, f) != 1) { err = "truncated LAZ point data"; return false; }
        if (table == -1) {   // written while streaming: the offset is in the last 8 bytes
            fseeko(f, (off_t)fsize - 8, SEEK_SET);
            if (fread(&table, 8, 1, f) != 1) { err = "truncated LAZ chunk table"; return false; }
        }
        if (table < (int64_t)data_off + 8 || (uint64_t)table + 8 > fsize) { err = "bad LAZ chunk table offset"; return false; }
        fseeko(f, (off_t)table, SEEK_SET);
        uint32_t hdr[2];
        if (fread(hdr, 4, 2, f) != 2) { err = "truncated LAZ chunk table"; return false; }
        const uint32_t nchunks = hdr[1];
        const bool variable = v.chunk_size == 0xFFFFFFFFu;
        // a chunk holds at least one point, and fixed-size chunks exactly
        // ceil(npoints / chunk_size) of them: anything larger is a corrupt table
        // (and would size the vectors below from untrusted bytes)
        const uint64_t max_chunks = variable ? std::max<uint64_t>(npoints, 1)
                                             : (v.chunk_size ? (npoints + v.chunk_size - 1) / v.chunk_size : 0);
        if (nchunks > max_chunks) { err = "bad LAZ chunk count"; return false; }
        std::vector<uint8_t> tb((size_t)(fsize - (uint64_t)table - 8));
        if (!tb.empty() && fread(tb.data(), 1, tb.size(), f) != tb.size()) { err = "truncated LAZ chunk table"; return false; }
        Decoder d;
        d.init(tb.data(), tb.data() + tb.size());
        IntegerCompressor ic(false, 32, 2);
        ic.init();
        std::vector<uint64_t> sizes(nchunks), counts(nchunks);
        int32_t pc = 0, ps = 0;
        for (uint32_t i = 0; i < nchunks; i++) {
            if (variable) counts[i] = (uint32_t)(pc = ic.decompress(d, pc, 0));
            sizes[i] = (uint32_t)(ps = ic.decompress(d, ps, 1));
        }
        uint64_t pos = data_off + 8, done = 0;
        chunk_start_.push_back(pos);
        for (uint32_t i = 0; i < nchunks; i++) {
            pos += sizes[i];
            chunk_start_.push_back(pos);
            const uint64_t c = std::min<uint64_t>(variable ? counts[i] : v.chunk_size, npoints - done);
            chunk_pts_.push_back(c);
            done += c;
        }
        if (pos > (uint64_t)table) { err = "LAZ chunk table beyond the point data"; return false; }
    }
    chunk_ = 0;
    in_chunk_ = chunk_n_ = 0;
    return true;
}

bool Reader::load_chunk(std::string& err) {
    if (chunk_ >= chunk_pts_.size()) { err = "LAZ point data ends before the point count"; return false; }
    const uint64_t a = chunk_start_[chunk_], b = chunk_start_[chunk_ + 1];
    buf_.resize((size_t)(b - a));
    fseeko(f_, (off_t)a, SEEK_SET);
    if (!buf_.empty() && fread(buf_.data(), 1, buf_.size(), f_) != buf_.size()) { err = "truncated LAZ chunk"; return false; }
    chunk_n_ = chunk_pts_[chunk_];
    in_chunk_ = 0;
    dec_->first = true;
    chunk_++;
    return true;
}

uint64_t Reader::read(uint8_t* out, uint64_t m, std::string& err) {
    uint64_t got = 0;
    PointDecoder& P = *dec_;
    while (got < m && left_ > 0) {
        if (in_chunk_ == chunk_n_ && !load_chunk(err)) return got;
        uint8_t* rec = out + got * rec_;
        if (!P.layered.empty()) {
            if (P.first) {
                // layered chunk: the first point raw, its point count, every
                // layer's size, then the layers in that order
                size_t o = rec_ + 4;
                uint32_t nl = 0;
                for (auto& it : P.layered) nl += it->layers();
                if (buf_.size() < o + 4ull * nl) { err = "truncated LAZ chunk"; return got; }
                memcpy(rec, buf_.data(), rec_);
                std::vector<uint32_t> ln(nl);
                memcpy(ln.data(), buf_.data() + o, 4ull * nl);
                o += 4ull * nl;
                std::vector<const uint8_t*> lp(nl);
                for (uint32_t i = 0; i < nl; i++) {
                    if (o + ln[i] > buf_.size()) { err = "truncated LAZ chunk"; return got; }
                    lp[i] = buf_.data() + o;
                    o += ln[i];
                }
                size_t io = 0;
                uint32_t li = 0;
                for (size_t i = 0; i < P.layered.size(); i++) {
                    P.layered[i]->init_dec(rec + io, P.ctx, lp.data() + li, ln.data() + li);
                    li += P.layered[i]->layers();
                    io += P.sizes[i];
                }
                P.first = false;
            } else {
                size_t io = 0;
                for (size_t i = 0; i < P.layered.size(); i++) {
                    P.layered[i]->read(rec + io, P.ctx);
                    io += P.sizes[i];
                    if (P.layered[i]->overrun()) { err = "corrupt LAZ chunk"; return got; }
                }
            }
        } else if (P.first) {   // the chunk's first point is stored raw, then the coder starts
            if (buf_.size() < rec_) { err = "truncated LAZ chunk"; return got; }
            memcpy(rec, buf_.data(), rec_);
            size_t o = 0;
            for (size_t i = 0; i < P.codecs.size(); i++) {
                P.codecs[i]->init(rec + o);
                o += P.sizes[i];
            }
            P.dec.init(buf_.data() + rec_, buf_.data() + buf_.size());
            P.first = false;
        } else {
            size_t o = 0;
            for (size_t i = 0; i < P.codecs.size(); i++) {
                P.codecs[i]->read(P.dec, rec + o);
                o += P.sizes[i];
            }
            if (P.dec.overrun) {   // read past the chunk's bytes (the encoder pads them): corrupt or cut
                err = "corrupt LAZ chunk";
                return got;
            }
        }
        in_chunk_++;
        got++;
        left_--;
    }
    return got;
}

std::vector<uint8_t> compress(const uint8_t* recs, uint64_t n, uint16_t rec, const std::vector<Item>& items,
                              uint32_t chunk_size) {
    std::vector<std::unique_ptr<ItemCodec>> codecs;
    std::vector<std::unique_ptr<LayeredItem>> layered;
    std::string err;
    const bool lay = is_layered(items);
    if (lay ? !make_layered(items, true, layered, err) : !make_codecs(items, true, codecs, err))
        throw std::runtime_error(err);
    std::vector<uint8_t> out(8, 0);   // chunk table offset, filled below
    std::vector<uint64_t> sizes;
    for (uint64_t c0 = 0; c0 < n && lay; c0 += chunk_size) {
        const uint64_t c1 = std::min<uint64_t>(n, c0 + chunk_size);
        const size_t start = out.size();
        out.insert(out.end(), recs + c0 * rec, recs + (c0 + 1) * rec);   // first point raw
        const uint32_t count = (uint32_t)(c1 - c0);
        out.insert(out.end(), reinterpret_cast<const uint8_t*>(&count), reinterpret_cast<const uint8_t*>(&count) + 4);
        uint32_t ctx = 0;
        size_t o = 0;
        for (size_t i = 0; i < layered.size(); i++) {
            layered[i]->init_enc(recs + c0 * rec + o, ctx);
            o += items[i].size;
        }
        for (uint64_t p = c0 + 1; p < c1; p++) {
            o = 0;
            for (size_t i = 0; i < layered.size(); i++) {
                layered[i]->write(recs + p * rec + o, ctx);
                o += items[i].size;
            }
        }
        std::vector<std::vector<uint8_t>> ls;
        for (auto& it : layered) it->finish(ls);
        for (auto& l : ls) {
            const uint32_t sz = (uint32_t)l.size();
            out.insert(out.end(), reinterpret_cast<const uint8_t*>(&sz), reinterpret_cast<const uint8_t*>(&sz) + 4);
        }
        for (auto& l : ls) out.insert(out.end(), l.begin(), l.end());
        sizes.push_back(out.size() - start);
    }
    for (uint64_t c0 = 0; c0 < n && !lay; c0 += chunk_size) {
        const uint64_t c1 = std::min<uint64_t>(n, c0 + chunk_size);
        const size_t start = out.size();
        out.insert(out.end(), recs + c0 * rec, recs + (c0 + 1) * rec);   // first point raw
        size_t o = 0;
        for (size_t i = 0; i < codecs.size(); i++) {
            codecs[i]->init(recs + c0 * rec + o);
            o += items[i].size;
        }
        std::vector<uint8_t> stream;
        Encoder e;
        e.init(&stream);
        for (uint64_t p = c0 + 1; p < c1; p++) {
            o = 0;
            for (size_t i = 0; i < codecs.size(); i++) {
                codecs[i]->write(e, recs + p * rec + o);
                o += items[i].size;
            }
        }
        e.done();
        out.insert(out.end(), stream.begin(), stream.end());
        sizes.push_back(out.size() - start);
    }
    const int64_t table = (int64_t)out.size();
    memcpy(out.data(), &table, 8);
    const uint32_t hdr[2] = {0, (uint32_t)sizes.size()};
    out.insert(out.end(), reinterpret_cast<const uint8_t*>(hdr), reinterpret_cast<const uint8_t*>(hdr) + 8);
    std::vector<uint8_t> tstream;
    Encoder e;
    e.init(&tstream);
    IntegerCompressor ic(true, 32, 2);
    ic.init();
    int32_t ps = 0;
    for (uint64_t s : sizes) {
        ic.compress(e, ps, (int32_t)s, 1);
        ps = (int32_t)s;
    }
    e.done();
    out.insert(out.end(), tstream.begin(), tstream.end());
    return out;
}

}  // namespace laz
}  // namespace pcc
