// cs_ddz_table.cpp -- the DouDizhu action table: compiled into the library from ddz_actions.bin (tools/gen_ddz_table.py)
// and expanded once per handle into the device lookup tables of cs_doudizhu.h (groups, per-dword group ranges).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <string>
#include <vector>
#include "cs_doudizhu.h"

#ifndef CS_DDZ_TABLE_FILE
#error "CS_DDZ_TABLE_FILE must name ddz_actions.bin (set by the Makefile)"
#endif

__asm__(".section .rodata\n"
        ".balign 16\n"
        ".local cs_ddz_blob\n"
        "cs_ddz_blob:\n"
        ".incbin \"" CS_DDZ_TABLE_FILE "\"\n"
        ".local cs_ddz_blob_end\n"
        "cs_ddz_blob_end:\n"
        ".previous\n");
extern "C" const unsigned char cs_ddz_blob[];
extern "C" const unsigned char cs_ddz_blob_end[];

namespace cs {
namespace ddz {

// Expands the compiled table into the host image of the device tables (cnt | gid | grp | drange, one allocation's
// layout, offsets in *off) and the scalar fields of *tab; returns an error message or "" on success. Host code only
// (the sanitizer driver, tools/san_driver.cpp, runs it without a GPU).
std::string table_build_host(std::vector<uint8_t>& host, size_t off[4], Tab* tab)
{
    const size_t size = (size_t)(cs_ddz_blob_end - cs_ddz_blob);
    if (size < 16 || memcmp(cs_ddz_blob, "DDZT", 4) != 0) return "doudizhu action table missing from the library";
    uint32_t na, pass;
    memcpy(&na, cs_ddz_blob + 4, 4);
    memcpy(&pass, cs_ddz_blob + 8, 4);
    if (na != (uint32_t)NA || pass != (uint32_t)PASS || size != 16 + (size_t)na * 12)   // + the host-only tc_order
        return "doudizhu action table has an unexpected size";
    std::vector<uint64_t> cnt(NA);
    memcpy(cnt.data(), cs_ddz_blob + 16, (size_t)NA * 8);
    const uint8_t* type = cs_ddz_blob + 16 + (size_t)NA * 8;
    const uint8_t* weight = type + NA;

    // solo ids 0..14 are the 15 single ranks in order (the fallback of an illegal leading action relies on it)
    for (int r = 0; r < 15; r++)
        if (cnt[r] != (1ull << (4 * r)) || type[r] != 0) return "doudizhu table: ids 0..14 are not the solos";
    // groups = maximal runs of equal (type, weight) over ids < PASS; every type one contiguous range, weights rising
    std::vector<uint16_t> gid(NA, 0);
    std::vector<uint32_t> grp((size_t)MAX_GROUPS * 4, 0);
    std::vector<int> gstart, gend, gtype;
    std::vector<int> type_lo(256, -1), type_hi(256, -1);
    for (int id = 0; id < PASS; id++) {
        const bool fresh = id == 0 || type[id] != type[id - 1] || weight[id] != weight[id - 1];
        if (fresh) {
            if (id > 0 && type[id] == type[id - 1] && weight[id] < weight[id - 1])
                return "doudizhu table: weights fall inside a type";
            if (type_lo[type[id]] >= 0 && (id == 0 || type[id] != type[id - 1]))
                return "doudizhu table: a type is not one contiguous id range";
            if (type_lo[type[id]] < 0) type_lo[type[id]] = id;
            gstart.push_back(id);
            gend.push_back(id + 1);
            gtype.push_back(type[id]);
        } else {
            gend.back() = id + 1;
        }
        type_hi[type[id]] = id + 1;
        gid[id] = (uint16_t)(gstart.size() - 1);
    }
    gid[PASS] = 0;
    const int ng = (int)gstart.size();
    if (ng > MAX_GROUPS) return "doudizhu table: too many (type, weight) groups";
    for (int g = 0; g < ng; g++) {
        uint64_t mn = ~0ull;
        for (int id = gstart[g]; id < gend[g]; id++) {
            uint64_t m = 0;
            for (int r = 0; r < 15; r++) {
                const uint64_t a = (mn >> (4 * r)) & 15, b = (cnt[id] >> (4 * r)) & 15;
                m |= (a < b ? a : b) << (4 * r);
            }
            mn = m;
        }
        uint32_t* e = &grp[(size_t)g * 4];
        e[0] = (uint32_t)mn;
        e[1] = (uint32_t)(mn >> 32);
        e[2] = (uint32_t)gstart[g] | ((uint32_t)gend[g] << 16);
        e[3] = (uint32_t)type_hi[gtype[g]] | ((uint32_t)gtype[g] << 16) | ((uint32_t)weight[gstart[g]] << 24);
    }
    std::vector<uint32_t> drange(ND, 0);
    for (int d = 0; d < ND; d++) {
        const int lo = 32 * d, hi = (32 * d + 31 < PASS - 1 ? 32 * d + 31 : PASS - 1);
        drange[d] = lo < PASS ? (uint32_t)gid[lo] | ((uint32_t)gid[hi] << 16) : 0u;
    }
    if (type_lo[TYPE_BOMB] < 0 || type_lo[TYPE_ROCKET] < 0 || type_hi[TYPE_ROCKET] != type_lo[TYPE_ROCKET] + 1)
        return "doudizhu table: bomb / rocket ranges not found";
    // the kernels compute the packed counts and groups of the simple ids (cs_doudizhu.h simple_cnt / simple_gid)
    const uint32_t blo = (uint32_t)type_lo[TYPE_BOMB], bg = gid[blo];
    if (type_hi[TYPE_BOMB] != (int)blo + 13 || type_lo[TYPE_ROCKET] != (int)blo + 13)
        return "doudizhu table: bombs and rocket are not 14 consecutive ids";
    for (uint32_t id = 0; id < (uint32_t)PASS; id++) {
        if (!simple_id(id, blo)) continue;
        if (cnt[id] != simple_cnt(id, blo) || gid[id] != simple_gid(id, blo, bg))
            return "doudizhu table: solo / pair / trio / bomb / rocket ids out of the kernels' layout";
    }

    // one device allocation: cnt | gid | grp | drange
    const size_t o_cnt = 0, o_gid = o_cnt + (size_t)NA * 8, o_grp = (o_gid + (size_t)NA * 2 + 255) & ~(size_t)255,
                 o_dr = o_grp + grp.size() * 4, total = o_dr + (size_t)ND * 4;
    host.assign(total, 0);
    memcpy(host.data() + o_cnt, cnt.data(), (size_t)NA * 8);
    memcpy(host.data() + o_gid, gid.data(), (size_t)NA * 2);
    memcpy(host.data() + o_grp, grp.data(), grp.size() * 4);
    memcpy(host.data() + o_dr, drange.data(), (size_t)ND * 4);
    off[0] = o_cnt; off[1] = o_gid; off[2] = o_grp; off[3] = o_dr;
    tab->ng = ng;
    tab->bomb_lo = type_lo[TYPE_BOMB];
    tab->bomb_hi = type_hi[TYPE_BOMB];
    tab->rocket = type_lo[TYPE_ROCKET];
    tab->bomb_g = (int32_t)bg;
    for (int k = 0; k <= MAX_GROUPS / 32; k++) tab->kfirst[k] = 32 * k < ng ? gstart[32 * k] : PASS;
    return "";
}

// Builds the device tables; returns an error message or "" on success. *dev owns one allocation.
std::string table_create(void** dev, Tab* tab)
{
    *dev = nullptr;
    std::vector<uint8_t> host;
    size_t off[4];
    const std::string err = table_build_host(host, off, tab);
    if (!err.empty()) return err;
    uint8_t* d = nullptr;
    if (hipMalloc((void**)&d, host.size()) != hipSuccess) return "hipMalloc (doudizhu action table)";
    if (hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return "hipMemcpy (doudizhu action table)";
    }
    *dev = d;
    tab->cnt = (const uint64_t*)(d + off[0]);
    tab->gid = (const uint16_t*)(d + off[1]);
    tab->grp = (const uint32_t*)(d + off[2]);
    tab->drange = (const uint32_t*)(d + off[3]);
    return "";
}

}  // namespace ddz
}  // namespace cs
