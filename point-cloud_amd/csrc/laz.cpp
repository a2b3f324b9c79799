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
        const uint32_t sym = d.symbol(m_used);
        if (sym & 1) c[0] = (uint16_t)u8_fold((int32_t)d.symbol(m_diff[0]) + (last[0] & 255));
        else c[0] = last[0] & 0xFF;
        if (sym & 2) c[0] |= (uint16_t)(u8_fold((int32_t)d.symbol(m_diff[1]) + (last[0] >> 8)) << 8);
        else c[0] |= last[0] & 0xFF00;
        if (sym & 64) {
            int32_t diff = (c[0] & 0xFF) - (last[0] & 0xFF);
            if (sym & 4) c[1] = (uint16_t)u8_fold((int32_t)d.symbol(m_diff[2]) + u8_clamp(diff + (last[1] & 255)));
            else c[1] = last[1] & 0xFF;
            if (sym & 16) {
                diff = (diff + ((c[1] & 0xFF) - (last[1] & 0xFF))) / 2;
                c[2] = (uint16_t)u8_fold((int32_t)d.symbol(m_diff[4]) + u8_clamp(diff + (last[2] & 255)));
            } else {
                c[2] = last[2] & 0xFF;
            }
            diff = (c[0] >> 8) - (last[0] >> 8);
            if (sym & 8) c[1] |= (uint16_t)(u8_fold((int32_t)d.symbol(m_diff[3]) + u8_clamp(diff + (last[1] >> 8))) << 8);
            else c[1] |= last[1] & 0xFF00;
            if (sym & 32) {
                diff = (diff + ((c[1] >> 8) - (last[1] >> 8))) / 2;
                c[2] |= (uint16_t)(u8_fold((int32_t)d.symbol(m_diff[5]) + u8_clamp(diff + (last[2] >> 8))) << 8);
            } else {
                c[2] |= last[2] & 0xFF00;
            }
        } else {
            c[1] = c[0];
            c[2] = c[0];
        }
        memcpy(last, c, 6);
        memcpy(item, c, 6);
    }
    void write(Encoder& e, const uint8_t* item) override {
        uint16_t c[3];
        memcpy(c, item, 6);
        uint32_t sym = ((last[0] & 0x00FF) != (c[0] & 0x00FF)) | (((last[0] & 0xFF00) != (c[0] & 0xFF00)) << 1) |
                       (((last[1] & 0x00FF) != (c[1] & 0x00FF)) << 2) | (((last[1] & 0xFF00) != (c[1] & 0xFF00)) << 3) |
                       (((last[2] & 0x00FF) != (c[2] & 0x00FF)) << 4) | (((last[2] & 0xFF00) != (c[2] & 0xFF00)) << 5) |
                       (((c[0] & 0x00FF) != (c[1] & 0x00FF) || (c[0] & 0x00FF) != (c[2] & 0x00FF) ||
                         (c[0] & 0xFF00) != (c[1] & 0xFF00) || (c[0] & 0xFF00) != (c[2] & 0xFF00)) << 6);
        e.symbol(m_used, sym);
        if (sym & 1) e.symbol(m_diff[0], u8_fold((c[0] & 255) - (last[0] & 255)));
        if (sym & 2) e.symbol(m_diff[1], u8_fold((c[0] >> 8) - (last[0] >> 8)));
        if (sym & 64) {
            int32_t diff = (c[0] & 0xFF) - (last[0] & 0xFF);
            if (sym & 4) e.symbol(m_diff[2], u8_fold((c[1] & 255) - u8_clamp(diff + (last[1] & 255))));
            if (sym & 16) {
                diff = (diff + ((c[1] & 0xFF) - (last[1] & 0xFF))) / 2;
                e.symbol(m_diff[4], u8_fold((c[2] & 255) - u8_clamp(diff + (last[2] & 255))));
            }
            diff = (c[0] >> 8) - (last[0] >> 8);
            if (sym & 8) e.symbol(m_diff[3], u8_fold((c[1] >> 8) - u8_clamp(diff + (last[1] >> 8))));
            if (sym & 32) {
                diff = (diff + ((c[1] >> 8) - (last[1] >> 8))) / 2;
                e.symbol(m_diff[5], u8_fold((c[2] >> 8) - u8_clamp(diff + (last[2] >> 8))));
            }
        }
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

bool make_codecs(const std::vector<Item>& items, bool enc, std::vector<std::unique_ptr<ItemCodec>>& out,
                 std::string& err) {
    out.clear();
    for (const Item& it : items) {
        if (it.type == POINT10 && it.size == 20 && it.version == 2) out.emplace_back(new Point10(enc));
        else if (it.type == GPSTIME11 && it.size == 8 && it.version == 2) out.emplace_back(new Gps11(enc));
        else if (it.type == RGB12 && it.size == 6 && it.version == 2) out.emplace_back(new Rgb12(enc));
        else if (it.type == BYTE && it.size >= 1 && it.version == 2) out.emplace_back(new Bytes(enc, it.size));
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
    std::vector<uint16_t> sizes;
    Decoder dec;
    bool first = true;
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

bool items_for_format(uint8_t format, uint16_t rec, std::vector<Item>& items, std::string& err) {
    static const uint16_t base[4] = {20, 28, 26, 34};
    if (format > 3) { err = "LAZ point format " + std::to_string(format) + " (layered compression) is not supported"; return false; }
    if (rec < base[format]) { err = "point record shorter than its format"; return false; }
    items.clear();
    items.push_back({POINT10, 20, 2});
    if (format == 1 || format == 3) items.push_back({GPSTIME11, 8, 2});
    if (format == 2 || format == 3) items.push_back({RGB12, 6, 2});
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
    if (v.compressor != 1 && v.compressor != 2) {
        err = "LAZ compressor " + std::to_string(v.compressor) + " (layered, point formats 6-10) is not supported";
        return false;
    }
    uint32_t sum = 0;
    for (const Item& it : v.items) sum += it.size;
    if (sum != rec) { err = "LAZ items do not add up to the point record length"; return false; }
    dec_.reset(new PointDecoder());
    if (!make_codecs(v.items, false, dec_->codecs, err)) return false;
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
        std::vector<uint8_t> tb((size_t)(fsize - (uint64_t)table - 8));
        if (!tb.empty() && fread(tb.data(), 1, tb.size(), f) != tb.size()) { err = "truncated LAZ chunk table"; return false; }
        Decoder d;
        d.init(tb.data(), tb.data() + tb.size());
        IntegerCompressor ic(false, 32, 2);
        ic.init();
        std::vector<uint64_t> sizes(nchunks), counts(nchunks);
        const bool variable = v.chunk_size == 0xFFFFFFFFu;
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
            const uint64_t c = variable ? counts[i] : std::min<uint64_t>(v.chunk_size, npoints - done);
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
        if (P.first) {   // the chunk's first point is stored raw, then the coder starts
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
    std::string err;
    if (!make_codecs(items, true, codecs, err)) throw std::runtime_error(err);
    std::vector<uint8_t> out(8, 0);   // chunk table offset, filled below
    std::vector<uint64_t> sizes;
    for (uint64_t c0 = 0; c0 < n; c0 += chunk_size) {
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
