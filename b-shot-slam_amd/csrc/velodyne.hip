// velodyne.hip -- Velodyne data-packet decode on the GPU: 1206-byte
// HDL-32E / VLP-16 packets -> velodyne::Laser records -> rotations, the loop of the reference's
// VelodyneCapture::capturePCAP (include/VelodyneCapture.h:413-525).
//
// Every record (packet, firing, laser slot) decodes independently: one thread each, 32-byte
// records written as four 8-byte words. The reference's sequential state -- last_azimuth, the
// rotation split at `last_azimuth > azimuth` and the specifiedframe skip -- depends only on the
// previous record's azimuth, so it becomes a flag per record, an inclusive scan (rotation number of
// every record) and the list of rotation starts; which rotations the reference would have pushed
// follows on the host from that list (a rotation is pushed at the next split, the last one never).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"
#include "velodyne.h"

namespace bvk {

// HDL32ECapture / VLP16Capture vertical tables (include/VelodyneCapture.h:572, :534)
__constant__ double c_lut32[32] = {-30.67, -9.3299999, -29.33, -8.0, -28, -6.6700001, -26.67, -5.3299999,
                                   -25.33, -4.0, -24.0, -2.6700001, -22.67, -1.33, -21.33, 0.0,
                                   -20.0, 1.33, -18.67, 2.6700001, -17.33, 4.0, -16, 5.3299999,
                                   -14.67, 6.6700001, -13.33, 8.0, -12.0, 9.3299999, -10.67, 10.67};
__constant__ double c_lut16[16] = {-15.0, 1.0, -13.0, 3.0, -11.0, 5.0, -9.0, 7.0,
                                   -7.0, 9.0, -5.0, 11.0, -3.0, 13.0, -1.0, 15.0};

__device__ __forceinline__ unsigned rd16(const unsigned char* p) { return (unsigned)p[0] | ((unsigned)p[1] << 8); }

// packet layout (:86-110): 12 firings of 100 B (u16 block id, u16 rotational position, 32 x
// {u16 distance, u8 intensity}), u32 GPS time, u8 mode, u8 sensor type at byte 1205
__global__ void k_velo_decode(const unsigned char* __restrict__ pk, const long long* __restrict__ unixtime,
                              int nrec, int maxl, double* __restrict__ az_out,
                              unsigned long long* __restrict__ rec, int* __restrict__ err) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    const int p = k / 384, r = k - p * 384, f = r >> 5, li = r & 31;
    const unsigned char* P = pk + (size_t)p * 1206;
    if (r == 0 && P[1205] != 0x21 && P[1205] != 0x22) atomicOr(err, 1);  // assert (:453)
    const unsigned rot0 = rd16(P + 2), rot1 = rd16(P + 102), rotf = rd16(P + f * 100 + 2);
    // integer promotion of the uint16 positions, then / 2.0 (:461-466)
    const double interpolated = rot1 < rot0 ? ((int)(rot1 + 36000) - (int)rot0) / 2.0 : ((int)rot1 - (int)rot0) / 2.0;
    double azimuth = (double)rotf;
    if (li >= maxl) azimuth += interpolated;
    if (azimuth >= 36000) azimuth -= 36000;
    az_out[k] = azimuth;
    const int slot = li % maxl;
    const unsigned char* R = P + f * 100 + 4 + 3 * slot;
    const double vertical = maxl == 16 ? c_lut16[slot] : c_lut32[slot];
    unsigned long long* o = rec + 4 * (size_t)k;
    o[0] = (unsigned long long)__double_as_longlong(azimuth / 100.0);
    o[1] = (unsigned long long)__double_as_longlong(vertical);
    o[2] = (unsigned long long)(rd16(R) | ((unsigned)R[2] << 16) | ((unsigned)slot << 24));
    o[3] = (unsigned long long)unixtime[p];
}

// rotation split flags: last_azimuth (0.0 before the first record) > azimuth (:474-489)
__global__ void k_velo_flags(const double* __restrict__ az, int nrec, int* __restrict__ flag) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    flag[k] = (k == 0 ? 0.0 : az[k - 1]) > az[k] ? 1 : 0;
}

// starts[g - 1] = first record of rotation g (g >= 1); tot[0] = number of splits
__global__ void k_velo_starts(const int* __restrict__ flag, const int* __restrict__ scan, int nrec,
                              int* __restrict__ starts, int* __restrict__ tot) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nrec) return;
    if (flag[k]) starts[scan[k] - 1] = k;
    if (k == nrec - 1) tot[0] = scan[k];
}

}  // namespace bvk

namespace bsh {

struct VeloState {
    DBuf<unsigned char> pk, tmp;
    DBuf<long long> ut;
    DBuf<double> az;
    DBuf<int> flag, scan, starts, tot;
    DBuf<unsigned long long> rec;
    PinBuf<unsigned char> p_pk;
    PinBuf<long long> p_ut;
    PinBuf<int> p_starts;
};

void velo_free(VeloState* v) {
    if (!v) return;
    v->pk.release(); v->tmp.release(); v->ut.release(); v->az.release(); v->flag.release(); v->scan.release();
    v->starts.release(); v->tot.release(); v->rec.release(); v->p_pk.release(); v->p_ut.release();
    v->p_starts.release();
    delete v;
}

#define VCHK(call, what)                                \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return c->fail(what, e_); \
    } while (0)

// decode npk device-resident packets into d_rec (npk * 384 records, 4 words each); the pushed
// rotations as [start, start + count) ranges of d_rec (host arrays, rot_cap entries)
int velo_decode(bshot_ctx* c, const unsigned char* d_pk, const long long* d_ut, int npk, int max_lasers,
                int specified_frame, unsigned long long* d_rec, std::vector<int>& rot_start, std::vector<int>& rot_count) {
    rot_start.clear();
    rot_count.clear();
    if (npk <= 0) return BSHOT_OK;
    if (!c->velo) c->velo = new VeloState();
    VeloState& V = *c->velo;
    hipStream_t st = c->stream;
    const int nrec = npk * 384;
    VCHK(V.az.ensure(nrec), "velo alloc"); VCHK(V.flag.ensure(nrec), "velo alloc"); VCHK(V.scan.ensure(nrec), "velo alloc");
    VCHK(V.starts.ensure(nrec), "velo alloc"); VCHK(V.tot.ensure(4), "velo alloc"); VCHK(V.p_starts.ensure(nrec + 4), "velo alloc");
    size_t tb = 0;
    VCHK(rocprim::inclusive_scan(nullptr, tb, V.flag.p, V.scan.p, (size_t)nrec, rocprim::plus<int>(), st), "velo scan size");
    VCHK(V.tmp.ensure(tb), "velo alloc");
    VCHK(kfill(V.tot.p, 0, sizeof(int) * 4, st), "velo memset");
    const int B = 256, G = (nrec + B - 1) / B;
    const int sg = c->stage_begin(BSHOT_STAGE_PRE, st);
    bvk::k_velo_decode<<<G, B, 0, st>>>(d_pk, d_ut, nrec, max_lasers, V.az.p, d_rec, V.tot.p + 1);
    bvk::k_velo_flags<<<G, B, 0, st>>>(V.az.p, nrec, V.flag.p);
    tb = V.tmp.cap;
    VCHK(rocprim::inclusive_scan(V.tmp.p, tb, V.flag.p, V.scan.p, (size_t)nrec, rocprim::plus<int>(), st), "velo scan");
    bvk::k_velo_starts<<<G, B, 0, st>>>(V.flag.p, V.scan.p, nrec, V.starts.p, V.tot.p);
    c->stage_end(sg, st);
    VCHK(hipGetLastError(), "velo launch");
    VCHK(kcopy(V.p_starts.p, V.tot.p, sizeof(int) * 2, st), "velo D2H");
    VCHK(hipStreamSynchronize(st), "velo sync");
    const int splits = V.p_starts.p[0];
    if (V.p_starts.p[1]) return c->fail("velodyne decode: packet with a sensor type other than 0x21/0x22", BSHOT_EINVAL);
    std::vector<int> gs((size_t)splits + 1, 0);  // gs[g] = first record of rotation g
    if (splits > 0) {
        VCHK(hipMemcpy(gs.data() + 1, V.starts.p, sizeof(int) * splits, hipMemcpyDeviceToHost), "velo D2H starts");
    }
    c->resolve_events();
    // rotation g is pushed at split g + 1; with specifiedframe S > 0 rotations g < S are skipped and
    // the split that ends the skipping pushes the (empty) vector first (:474-489)
    if (specified_frame > 0) {
        if (splits >= specified_frame) {
            rot_start.push_back(gs[specified_frame]);
            rot_count.push_back(0);
            for (int g = specified_frame; g < splits; ++g) {
                rot_start.push_back(gs[g]);
                rot_count.push_back(gs[g + 1] - gs[g]);
            }
        }
    } else {
        for (int g = 0; g < splits; ++g) {
            rot_start.push_back(gs[g]);
            rot_count.push_back(gs[g + 1] - gs[g]);
        }
    }
    return BSHOT_OK;
}

}  // namespace bsh

extern "C" {

int bshot_velodyne_decode_device(bshot_ctx* c, const uint8_t* d_payloads, const int64_t* d_unixtime, int npk,
                                 int max_lasers, int specified_frame, bshot_laser* d_out, int32_t* rot_start,
                                 int32_t* rot_count, int rot_cap, int* n_rot) {
    if (!c || npk < 0 || (npk > 0 && (!d_payloads || !d_unixtime || !d_out)) || (max_lasers != 16 && max_lasers != 32) ||
        npk > (1 << 22) || rot_cap < 0 || (rot_cap > 0 && (!rot_start || !rot_count)))
        return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    std::vector<int> rs, rc;
    int e = bsh::velo_decode(c, d_payloads, reinterpret_cast<const long long*>(d_unixtime), npk, max_lasers,
                             specified_frame, reinterpret_cast<unsigned long long*>(d_out), rs, rc);
    if (e) return e;
    if (n_rot) *n_rot = (int)rs.size();
    if ((int)rs.size() > rot_cap) return c->fail("velodyne decode: rotation capacity too small", BSHOT_ECAP);
    for (size_t i = 0; i < rs.size(); ++i) {
        rot_start[i] = rs[i];
        rot_count[i] = rc[i];
    }
    return BSHOT_OK;
}

int bshot_velodyne_decode(bshot_ctx* c, const uint8_t* payloads, const int64_t* unixtime, int npk, int max_lasers,
                          int specified_frame, bshot_laser* out, int cap, int32_t* rot_start, int32_t* rot_count,
                          int rot_cap, int* n_rot, int* n_out) {
    if (!c || npk < 0 || (npk > 0 && (!payloads || !unixtime)) || (max_lasers != 16 && max_lasers != 32) ||
        npk > (1 << 22) || cap < 0 || (cap > 0 && !out) || rot_cap < 0 || (rot_cap > 0 && (!rot_start || !rot_count)))
        return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    if (n_out) *n_out = 0;
    if (n_rot) *n_rot = 0;
    if (npk == 0) return BSHOT_OK;
    if (!c->velo) c->velo = new bsh::VeloState();
    bsh::VeloState& V = *c->velo;
    const size_t nb = (size_t)npk * 1206;
    if (V.pk.ensure(nb) || V.p_pk.ensure(nb) || V.ut.ensure(npk) || V.p_ut.ensure(npk) ||
        V.rec.ensure((size_t)npk * 384 * 4))
        return c->fail("velodyne decode: alloc", BSHOT_EHIP);
    std::memcpy(V.p_pk.p, payloads, nb);
    std::memcpy(V.p_ut.p, unixtime, sizeof(int64_t) * npk);
    if (bsh::kcopy(V.pk.p, V.p_pk.p, nb, c->stream) ||
        bsh::kcopy(V.ut.p, V.p_ut.p, sizeof(int64_t) * npk, c->stream))
        return c->fail("velodyne decode: H2D", BSHOT_EHIP);
    std::vector<int> rs, rc;
    int e = bsh::velo_decode(c, V.pk.p, V.ut.p, npk, max_lasers, specified_frame, V.rec.p, rs, rc);
    if (e) return e;
    // the pushed rotations are consecutive records: one copy of their span
    int total = 0;
    for (int x : rc) total += x;
    if (n_rot) *n_rot = (int)rs.size();
    if (n_out) *n_out = total;
    if ((int)rs.size() > rot_cap || total > cap) return c->fail("velodyne decode: output capacity too small", BSHOT_ECAP);
    const int first = rs.empty() ? 0 : rs[0];
    for (size_t i = 0; i < rs.size(); ++i) {
        rot_start[i] = rs[i] - first;
        rot_count[i] = rc[i];
    }
    if (total > 0 && hipMemcpy(out, V.rec.p + 4 * (size_t)first, sizeof(bshot_laser) * (size_t)total,
                               hipMemcpyDeviceToHost) != hipSuccess)
        return c->fail("velodyne decode: D2H", BSHOT_EHIP);
    return BSHOT_OK;
}

}  // extern "C"
