// preprocess.hip -- point-cloud preprocessor on the GPU: Velodyne laser
// returns -> range image -> ground removal -> occluded-edge removal -> point cloud, the
// reference's myslam::Preprocessor::run (src/preprocess.cpp:217-226) without its std::maps.
//
// The reference keys three std::map<double, std::map<double, .>> (rimg, rmmap, selmap) by
// (azimuth, vertical) in radians. Here the range image is a sorted cell table in HBM:
//   * every laser l contributes two insertion events in the reference's order: e = 2l (its own
//     return, src/preprocess.cpp:54) and e = 2l + 1 (the synthetic vert_init_ entry, :55);
//   * two stable radix sorts (vertical key, then azimuth key, positions e as values) order the 2N
//     events by (azimuth, vertical, e): one run of equal keys per map entry ("cell"); the first
//     event of a run is the key std::map keeps, the last one the value that survives;
//   * a column (inner map) is a run of equal azimuth; its key is the azimuth of its lowest laser.
// Ground removal walks each column's cells in order (thread per column: the reference's
// sequential state machine, :72-164). Occlusion is one workgroup per vertical angle: the
// reference's "previous non-empty column" becomes a block max-scan, after which every column's
// test is independent (marks only turn 0 into 3, so their order does not matter) (:166-195).
// The write-out compacts the kept cells in map order (:197-215).
//
// Arithmetic follows the reference expression by expression (double geometry, float
// Eigen::Vector3f points, float asin, -ffp-contract=off). Scalars that depend only on parameters
// (2450/sin(vert_init), -2450/tan(vert_init), the vertical angles in radians) are computed on the
// host with the same libm as the reference; per-point sin/cos use the device's double libm.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "ctx.h"
#include "preprocess.h"

namespace bsh {

struct PreState {
    bshot_pre_params prm{};
    PreConsts K{};
    double syn_dist = 0;
    int n = 0, cells = 0, cols = 0;
    bool counts_ok = false;  // cells / cols copied back since the last read
    std::vector<double> vdeg, vj, rtab;
    int vinit_rank = 0;
    std::vector<unsigned char> h_sel;
    DBuf<bshot_laser> lasers;
    PinBuf<bshot_laser> p_lasers;
    DBuf<unsigned long long> vkey, vkey2, akey, akey2, cnt, scan;
    DBuf<unsigned> val, val2, perm;
    DBuf<int> cstart, colcell, colmin, tot, c_rm, c_sel, c_col, keep, offs, tab, ph0;
    DBuf<double> c_vr, c_dist, col_az, d_vj;
    DBuf<float4> pts;
    DBuf<int> colflag, colid, vrank, fbad;  // fast path
    DBuf<unsigned> fkey, fkey2;
    DBuf<double> d_rtab;
    PinBuf<double> p_rtab;
    PinBuf<int> p_fbad;
    int fast_runs = 0, general_runs = 0;
    DBuf<unsigned char> selm, tmp;
    DBuf<float> out;
    PinBuf<unsigned char> p_sel;
    PinBuf<double> p_vj;
    PinBuf<int> p_tot;
    const bshot_laser* d_lasers = nullptr;
};

void pre_free(PreState* p) {
    if (!p) return;
    p->lasers.release(); p->p_lasers.release();
    p->vkey.release(); p->vkey2.release(); p->akey.release(); p->akey2.release(); p->cnt.release(); p->scan.release();
    p->val.release(); p->val2.release(); p->perm.release();
    p->cstart.release(); p->colcell.release(); p->colmin.release(); p->tot.release(); p->c_rm.release();
    p->c_sel.release(); p->c_col.release(); p->keep.release(); p->offs.release(); p->tab.release(); p->ph0.release();
    p->c_vr.release(); p->c_dist.release(); p->col_az.release(); p->d_vj.release(); p->pts.release();
    p->colflag.release(); p->colid.release(); p->vrank.release(); p->fbad.release(); p->fkey.release();
    p->fkey2.release(); p->d_rtab.release(); p->p_rtab.release(); p->p_fbad.release();
    p->selm.release(); p->tmp.release(); p->out.release();
    p->p_sel.release(); p->p_vj.release(); p->p_tot.release();
    delete p;
}

}  // namespace bsh

namespace bpk {

constexpr double kPi = 3.1415926535897932384626433832795;  // CV_PI

// order-preserving 64-bit key of a double; +0 and -0 share one key (std::map equivalence)
__device__ __forceinline__ unsigned long long ordkey(double d) {
    unsigned long long u = (unsigned long long)__double_as_longlong(d);
    if ((u << 1) == 0) u = 0;
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double ev_vertical(const bshot_laser* L, unsigned e, double vinit) {
    return (e & 1u) ? vinit : L[e >> 1].vertical * kPi / 180.0;
}

// insertion events -> vertical keys (first sort)
__global__ void k_pre_vkeys(const bshot_laser* __restrict__ L, int n2, double vinit,
                            unsigned long long* __restrict__ vkey, unsigned* __restrict__ val) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n2) return;
    vkey[e] = ordkey(ev_vertical(L, (unsigned)e, vinit));
    val[e] = (unsigned)e;
}

// events in vertical order -> azimuth keys (second, stable sort)
__global__ void k_pre_akeys(const bshot_laser* __restrict__ L, const unsigned* __restrict__ val, int n2,
                            unsigned long long* __restrict__ akey) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n2) return;
    akey[s] = ordkey(L[val[s] >> 1].azimuth * kPi / 180.0);
}

// run starts: high word counts cells (equal azimuth and vertical), low word columns (equal azimuth)
__global__ void k_pre_flags(const bshot_laser* __restrict__ L, const unsigned* __restrict__ perm, int n2,
                            double vinit, unsigned long long* __restrict__ cnt) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n2) return;
    bool col = s == 0, cell = s == 0;
    if (s > 0) {
        const unsigned e = perm[s], ep = perm[s - 1];
        col = ordkey(L[e >> 1].azimuth * kPi / 180.0) != ordkey(L[ep >> 1].azimuth * kPi / 180.0);
        cell = col || ordkey(ev_vertical(L, e, vinit)) != ordkey(ev_vertical(L, ep, vinit));
    }
    cnt[s] = ((unsigned long long)(cell ? 1u : 0u) << 32) | (col ? 1u : 0u);
}

// fast-path test: lasers already in nondecreasing azimuth order (every rotation the capture
// pushes is, include/VelodyneCapture.h:474-489) and every vertical angle found in the rank table
// (the vertical table plus vert_init_, sorted, distinct). bad[0] = 1 when either fails.
// colflag[l] = 1 where a new azimuth starts; vrank[l] = rank of the laser's vertical.
__global__ void k_pre_check(const bshot_laser* __restrict__ L, int n, const double* __restrict__ rtab, int nr,
                            int* __restrict__ colflag, int* __restrict__ vrank, int* __restrict__ bad) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= n) return;
    const double az = L[l].azimuth * kPi / 180.0;
    bool b = !(az == az);
    int cf = 1;
    if (l > 0) {
        const unsigned long long k0 = ordkey(L[l - 1].azimuth * kPi / 180.0), k1 = ordkey(az);
        if (k1 < k0) b = true;
        cf = k1 != k0;
    }
    const double vr = L[l].vertical * kPi / 180.0;
    int lo = 0, hi = nr;  // first rank with rtab >= vr
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rtab[mid] < vr) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= nr || !(rtab[lo] == vr)) b = true;
    colflag[l] = cf;
    vrank[l] = lo;
    if (b) atomicOr(bad, 1);
}

// fast-path keys: (column << 9 | vertical rank) per event; one stable 32-bit sort then orders the
// events by (azimuth, vertical, e) exactly as the two 64-bit sorts do
__global__ void k_pre_fkeys(const int* __restrict__ colid, const int* __restrict__ vrank, int vinit_rank, int n2,
                            unsigned* __restrict__ key, unsigned* __restrict__ val) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n2) return;
    const int l = e >> 1;
    key[e] = ((unsigned)(colid[l] - 1) << 9) | (unsigned)((e & 1) ? vinit_rank : vrank[l]);
    val[e] = (unsigned)e;
}

// cell / column starts and totals (tot[0] cells, tot[1] columns)
__global__ void k_pre_starts(const unsigned long long* __restrict__ cnt, const unsigned long long* __restrict__ scan,
                             int n2, int* __restrict__ cstart, int* __restrict__ colcell, int* __restrict__ tot) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n2) return;
    const unsigned long long f = cnt[s], sc = scan[s];
    const int m = (int)(sc >> 32) - 1, c = (int)(sc & 0xFFFFFFFFu) - 1;
    if (f >> 32) cstart[m] = s;
    if (f & 0xFFFFFFFFu) colcell[c] = m;
    if (s == n2 - 1) {
        tot[0] = m + 1;
        tot[1] = c + 1;
        cstart[m + 1] = n2;
        colcell[c + 1] = m + 1;
    }
}

// one thread per cell: key (first event of the run), surviving value (last event), selection flag
// of the last real return (-1: selmap has no entry), column. Every laser of a column adds an event
// to the column's vert_init_ cell and each such run ends with a synthetic event, so the first event
// of that run belongs to the column's lowest laser: its azimuth is the column's key (colmin).
__global__ void k_pre_cells(const bshot_laser* __restrict__ L, const unsigned* __restrict__ perm,
                            const unsigned long long* __restrict__ scan, const int* __restrict__ cstart,
                            const unsigned char* __restrict__ selm, const int* __restrict__ tot, double vinit,
                            double syn_dist, int n2, double* __restrict__ c_vr, double* __restrict__ c_dist,
                            int* __restrict__ c_rm, int* __restrict__ c_sel, int* __restrict__ c_col,
                            int* __restrict__ colmin) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n2 || m >= tot[0]) return;
    const int s0 = cstart[m], s1 = cstart[m + 1] - 1;
    const unsigned e0 = perm[s0], e1 = perm[s1];
    c_vr[m] = ev_vertical(L, e0, vinit);
    if (e1 & 1u) {
        c_dist[m] = syn_dist;  // rimg[az][vert_init_] = 2450/sin(vert_init_), rmmap = 1 (:55, :57)
        c_rm[m] = 1;
    } else {
        c_dist[m] = static_cast<double>(L[e1 >> 1].distance) * 2;  // (:45)
        c_rm[m] = 0;
    }
    int sel = -1;
    for (int s = s1; s >= s0; --s) {
        const unsigned e = perm[s];
        if (!(e & 1u)) {
            sel = selm ? (int)selm[e >> 1] : 1;
            break;
        }
    }
    c_sel[m] = sel;
    const int col = (int)(scan[s0] & 0xFFFFFFFFu) - 1;
    c_col[m] = col;
    if (e1 & 1u) colmin[col] = (int)(e0 >> 1);
}

// per cell: the point the reference builds from it (double geometry, float Vector3f) and its
// self-car test (src/preprocess.cpp:92-95, :147-152; the same point as writePointCloud's, :206-209)
__global__ void k_pre_pts(const double* __restrict__ c_vr, const double* __restrict__ c_dist,
                          const int* __restrict__ c_col, const double* __restrict__ col_az, const int* __restrict__ tot,
                          int n2, float4* __restrict__ pts) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n2 || m >= tot[0]) return;
    const double vr = c_vr[m], dist = c_dist[m], az = col_az[c_col[m]];
    const double cv = cos(vr);
    const double x = dist * cv * sin(az);
    const double y = dist * cv * cos(az);
    const double z = dist * sin(vr);
    const bool selfcar = x <= 820 && x >= -820 && y <= 1300 && y >= -1800 && z <= 100 && z >= -2000;
    pts[m] = make_float4((float)x, (float)y, (float)z, selfcar ? 1.f : 0.f);
}

// column keys: the azimuth of the column's lowest laser
__global__ void k_pre_colaz(const bshot_laser* __restrict__ L, const int* __restrict__ colmin,
                            const int* __restrict__ tot, int n2, double* __restrict__ col_az) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n2 || c >= tot[1]) return;
    col_az[c] = L[colmin[c]].azimuth * kPi / 180.0;
}

struct F3 {
    float x, y, z;
};
__device__ __forceinline__ float f3norm(F3 a) { return sqrtf((a.x * a.x + a.y * a.y) + a.z * a.z); }

// removeGround (src/preprocess.cpp:72-164): one thread per column, the reference's state machine
// over the column's cells in vertical order (the first cell is skipped, :87-90); the points and
// self-car tests come precomputed per cell (k_pre_pts)
__global__ void k_pre_ground(const int* __restrict__ colcell, const int* __restrict__ tot, int n2, PreConsts K,
                             const double* __restrict__ c_dist, const float4* __restrict__ pts,
                             const double* __restrict__ col_az, int* __restrict__ c_rm) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n2 || c >= tot[1]) return;
    const double az = col_az[c];
    bool lost_pt = false, set_th_pt = false, prev_is_ground = true;
    const double x_0 = K.init_r * sin(az);  // (-2450/tan(vert_init_)) * sin(col.first)
    const double y_0 = K.init_r * cos(az);
    const double z_0 = -2450;
    F3 p_prev{(float)x_0, (float)y_0, (float)z_0};
    F3 p_th = p_prev;
    const int m1 = colcell[c + 1];
    for (int m = colcell[c] + 1; m < m1; ++m) {
        const double dist = c_dist[m];
        const float4 pc = pts[m];
        const F3 p_curr{pc.x, pc.y, pc.z};
        const F3 d{p_curr.x - p_prev.x, p_curr.y - p_prev.y, p_curr.z - p_prev.z};
        // asin(float) * 180 is float arithmetic; the division by CV_PI promotes to double (:95)
        const double grad = (double)(asinf((p_curr.z - p_prev.z) / f3norm(d)) * 180.0f) / kPi;
        const float prev_norm = f3norm(p_prev);
        int rm = c_rm[m];
        if (prev_is_ground && (grad > K.grad_th || dist == 0 || dist < prev_norm)) {
            set_th_pt = true;
            p_th = p_prev;
        }
        if (prev_is_ground) {
            if (grad < K.grad_th && !lost_pt) {
                rm = 1;
            } else {
                rm = 0;
                prev_is_ground = false;
            }
        } else if (p_curr.z < K.lowpt_th && grad < K.grad_th) {
            rm = 1;
            prev_is_ground = true;
            set_th_pt = false;
        }
        if (dist == 0) {
            rm = 1;
            lost_pt = true;
            prev_is_ground = false;
        } else {
            lost_pt = false;
        }
        if (dist < prev_norm && dist != 0) {
            rm = 0;
            prev_is_ground = false;
        }
        if (set_th_pt && (p_curr.z - p_th.z) < K.height_th && p_curr.z < p_prev.z) {
            set_th_pt = false;
            rm = 1;
            prev_is_ground = true;
        }
        if (pc.w != 0.f) rm = 2;  // self-car box (:147-152)
        c_rm[m] = rm;
        p_prev = p_curr;
    }
}

// occlusion lookup: tab[col * J + j] = the cell of column col at vertical angle j (or -1)
__global__ void k_pre_tab_clear(int* __restrict__ tab, const int* __restrict__ tot, int J) {
    const size_t total = (size_t)tot[1] * J;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        tab[i] = -1;
}
__global__ void k_pre_table(const double* __restrict__ c_vr, const int* __restrict__ c_col,
                            const int* __restrict__ tot, int n2, const double* __restrict__ vj, int J,
                            int* __restrict__ tab) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n2 || m >= tot[0]) return;
    const double v = c_vr[m];
    for (int j = 0; j < J; ++j)
        if (vj[j] == v) tab[(size_t)c_col[m] * J + j] = m;
}

// removeOccluded (src/preprocess.cpp:166-195) for vertical angle j = blockIdx.x. The reference's
// prev_hor for column c >= 1 is the last column in [1, c) with a non-zero range at this angle, else
// column 0: a block max-scan of each thread's last such column. ph0[j] records a mark the
// reference puts on a column-0 entry that rmmap did not hold (operator[] inserted it).
__global__ void __launch_bounds__(256) k_pre_occl(const int* __restrict__ tab, int J, const int* __restrict__ tot,
                                                   const double* __restrict__ c_dist, const double* __restrict__ col_az,
                                                   PreConsts K, int* __restrict__ c_rm, int* __restrict__ ph0) {
    __shared__ int sc[256];
    const int j = blockIdx.x, t = threadIdx.x;
    const int C = tot[1];
    const int per = (C + 255) / 256;
    const int b = t * per, e = min(C, b + per);
    int last = -1;
    for (int c = max(b, 1); c < e; ++c) {
        const int m = tab[(size_t)c * J + j];
        if (m >= 0 && c_dist[m] != 0) last = c;
    }
    sc[t] = last;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const int v = t >= off ? sc[t - off] : -1;
        __syncthreads();
        sc[t] = max(sc[t], v);
        __syncthreads();
    }
    int prev = t > 0 ? sc[t - 1] : -1;
    if (prev < 0) prev = 0;
    for (int c = max(b, 1); c < e; ++c) {
        const int m = tab[(size_t)c * J + j];
        const double d = m >= 0 ? c_dist[m] : 0.0;
        if (d == 0) continue;
        const int mp = tab[(size_t)prev * J + j];
        const double d_dist = d - (mp >= 0 ? c_dist[mp] : 0.0);
        const double d_hor = col_az[c] - col_az[prev];
        if (fabs(d_dist) > K.dist_th && fabs(d_hor) < K.angdiff_th) {
            if (d_dist > 0) {
                if (c_rm[m] == 0) c_rm[m] = 3;
            } else if (mp >= 0) {
                if (c_rm[mp] == 0) c_rm[mp] = 3;
            } else {
                ph0[j] = 1;
            }
        }
        prev = c;
    }
}

// writePointCloud (src/preprocess.cpp:197-215): keep flags, then the compacting write
__global__ void k_pre_keep(const double* __restrict__ c_vr, const double* __restrict__ c_dist,
                           const int* __restrict__ c_rm, const int* __restrict__ c_sel, const int* __restrict__ tot,
                           int n2, double vinit, int save_sel, int* __restrict__ keep) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n2) return;
    int k = 0;
    if (m < tot[0]) k = c_dist[m] != 0 && c_vr[m] != vinit && c_rm[m] == 0 && c_sel[m] == save_sel;
    keep[m] = k;
}

__global__ void k_pre_write(const float4* __restrict__ pts, const int* __restrict__ keep,
                            const int* __restrict__ offs, const int* __restrict__ tot, int n2, int cap,
                            float* __restrict__ xyz, int* __restrict__ n_out) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n2 || m >= tot[0]) return;
    const int o = offs[m];
    if (m == tot[0] - 1) *n_out = o + keep[m];
    if (!keep[m] || o >= cap) return;
    const float4 p = pts[m];
    xyz[3 * (size_t)o] = p.x;
    xyz[3 * (size_t)o + 1] = p.y;
    xyz[3 * (size_t)o + 2] = p.z;
}

}  // namespace bpk

namespace bsh {

#define PCHK(call, what)                                \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return c->fail(what, e_); \
    } while (0)

// reference selection semantics (src/preprocess.cpp:59-66 with setSelectedPoints' sort, :25-28):
// laser i is selected when it equals the next unmatched entry of the sorted list
static void selection_mask(const int32_t* sel, int nsel, int n, std::vector<unsigned char>& mask) {
    std::vector<int32_t> s(sel, sel + nsel);
    std::sort(s.begin(), s.end());
    mask.assign((size_t)n, 0);
    size_t k = 0;
    for (int i = 0; i < n; ++i)
        if (k < s.size() && s[k] == i) {
            mask[i] = 1;
            ++k;
        }
}

static PreState& pre_state(bshot_ctx* c) {
    if (!c->prep) c->prep = new PreState();
    return *c->prep;
}

int pre_stage_lasers(bshot_ctx* c, const bshot_laser* lasers, int n, const bshot_laser** d_out) {
    PreState& P = pre_state(c);
    *d_out = nullptr;
    if (n <= 0) return BSHOT_OK;
    PCHK(P.lasers.ensure(n), "pre alloc lasers");
    PCHK(P.p_lasers.ensure(n), "pre alloc lasers");
    std::memcpy(P.p_lasers.p, lasers, sizeof(bshot_laser) * (size_t)n);
    PCHK(kcopy(P.lasers.p, P.p_lasers.p, sizeof(bshot_laser) * (size_t)n, c->stream),
         "pre H2D lasers");
    *d_out = P.lasers.p;
    return BSHOT_OK;
}

// readFrame (src/preprocess.cpp:38-70): range-image cells of the laser returns (device-resident)
int pre_read(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
             const bshot_pre_params* prm, const int32_t* sel, int nsel) {
    PreState& P = pre_state(c);
    hipStream_t st = c->stream;
    bshot_pre_params pp;
    if (prm) pp = *prm;
    else bshot_pre_default_params(&pp);
    P.prm = pp;
    P.n = n > 0 ? n : 0;
    P.d_lasers = d_lasers;
    // vertAngle_ sorted (setVerticalAngles, :30-33), radians as removeOccluded computes them (:169)
    P.vdeg.assign(vert_deg, vert_deg + (vert_deg ? nv : 0));
    std::sort(P.vdeg.begin(), P.vdeg.end());
    const int J = (int)P.vdeg.size();
    P.vj.resize(J);
    for (int j = 0; j < J; ++j) P.vj[j] = P.vdeg[j] * bpk::kPi / 180.0;
    // fast-path rank table: the table's angles and vert_init_, sorted, equal values merged (+-0 too)
    P.rtab = P.vj;
    P.rtab.push_back(pp.vert_init);
    std::sort(P.rtab.begin(), P.rtab.end());
    P.rtab.erase(std::unique(P.rtab.begin(), P.rtab.end(), [](double a, double b) { return a == b; }), P.rtab.end());
    P.vinit_rank = (int)(std::lower_bound(P.rtab.begin(), P.rtab.end(), pp.vert_init) - P.rtab.begin());
    P.K.grad_th = 45;
    P.K.lowpt_th = pp.lowpt_th;
    P.K.height_th = 500;
    P.K.dist_th = 3000;
    P.K.angdiff_th = 1.0 * bpk::kPi / 180.0;
    P.K.init_r = -2450 / std::tan(pp.vert_init);
    P.syn_dist = 2450 / std::sin(pp.vert_init);
    P.cells = 0;
    P.cols = 0;
    P.counts_ok = n <= 0;
    if (n <= 0) return BSHOT_OK;
    const int n2 = 2 * n;
    PCHK(P.vkey.ensure(n2), "pre alloc"); PCHK(P.vkey2.ensure(n2), "pre alloc");
    PCHK(P.akey.ensure(n2), "pre alloc"); PCHK(P.akey2.ensure(n2), "pre alloc");
    PCHK(P.val.ensure(n2), "pre alloc"); PCHK(P.val2.ensure(n2), "pre alloc"); PCHK(P.perm.ensure(n2), "pre alloc");
    PCHK(P.cnt.ensure(n2), "pre alloc"); PCHK(P.scan.ensure(n2), "pre alloc");
    PCHK(P.cstart.ensure(n2 + 1), "pre alloc"); PCHK(P.colcell.ensure(n2 + 1), "pre alloc");
    PCHK(P.colmin.ensure(n2), "pre alloc"); PCHK(P.tot.ensure(4), "pre alloc");
    PCHK(P.c_vr.ensure(n2), "pre alloc"); PCHK(P.c_dist.ensure(n2), "pre alloc");
    PCHK(P.c_rm.ensure(n2), "pre alloc"); PCHK(P.c_sel.ensure(n2), "pre alloc"); PCHK(P.c_col.ensure(n2), "pre alloc");
    PCHK(P.col_az.ensure(n2), "pre alloc"); PCHK(P.keep.ensure(n2), "pre alloc"); PCHK(P.offs.ensure(n2), "pre alloc");
    PCHK(P.pts.ensure(n2), "pre alloc");
    PCHK(P.ph0.ensure(J > 0 ? J : 1), "pre alloc"); PCHK(P.d_vj.ensure(J > 0 ? J : 1), "pre alloc");
    PCHK(P.p_tot.ensure(4), "pre alloc");
    size_t need = 0, tb = 0;
    PCHK(rocprim::radix_sort_pairs(nullptr, tb, P.vkey.p, P.vkey2.p, P.val.p, P.val2.p, (unsigned)n2, 0, 64, st),
         "pre sort size");
    need = std::max(need, tb);
    tb = 0;
    PCHK(rocprim::inclusive_scan(nullptr, tb, P.cnt.p, P.scan.p, (size_t)n2, rocprim::plus<unsigned long long>(), st),
         "pre scan size");
    need = std::max(need, tb);
    tb = 0;
    PCHK(rocprim::exclusive_scan(nullptr, tb, P.keep.p, P.offs.p, 0, (size_t)n2, rocprim::plus<int>(), st),
         "pre scan size");
    need = std::max(need, tb);
    tb = 0;
    PCHK(rocprim::radix_sort_pairs(nullptr, tb, (unsigned*)nullptr, (unsigned*)nullptr, P.val.p, P.perm.p, (unsigned)n2, 0,
                                   32, st),
         "pre sort size");
    need = std::max(need, tb);
    tb = 0;
    PCHK(rocprim::inclusive_scan(nullptr, tb, (int*)nullptr, (int*)nullptr, (size_t)n, rocprim::plus<int>(), st),
         "pre scan size");
    need = std::max(need, tb);
    PCHK(P.tmp.ensure(need), "pre alloc tmp");
    const unsigned char* selm = nullptr;
    if (pp.have_sel_list) {
        selection_mask(sel, sel ? nsel : 0, n, P.h_sel);
        PCHK(P.selm.ensure(n), "pre alloc sel");
        PCHK(P.p_sel.ensure(n), "pre alloc sel");
        std::memcpy(P.p_sel.p, P.h_sel.data(), (size_t)n);
        PCHK(kcopy(P.selm.p, P.p_sel.p, (size_t)n, st), "pre H2D sel");
        selm = P.selm.p;
    }
    if (J > 0) {
        PCHK(P.p_vj.ensure(J), "pre alloc");
        std::memcpy(P.p_vj.p, P.vj.data(), sizeof(double) * J);
        PCHK(kcopy(P.d_vj.p, P.p_vj.p, sizeof(double) * J, st), "pre H2D vj");
    }
    const int sg = c->stage_begin(BSHOT_STAGE_PRE, st);
    const int B = 256, G = (n2 + B - 1) / B;
    // fast path (azimuth-ordered lasers whose verticals are all in the table): one 32-bit sort of
    // (column, vertical rank); otherwise two stable 64-bit sorts (vertical, then azimuth)
    bool fast = false;
    if (c->opt_pre_fast && !P.rtab.empty() && P.rtab.size() <= 512 && n < (1 << 22)) {
        const int nr = (int)P.rtab.size();
        PCHK(P.colflag.ensure(n), "pre alloc"); PCHK(P.colid.ensure(n), "pre alloc"); PCHK(P.vrank.ensure(n), "pre alloc");
        PCHK(P.fbad.ensure(1), "pre alloc"); PCHK(P.p_fbad.ensure(1), "pre alloc");
        PCHK(P.d_rtab.ensure(nr), "pre alloc"); PCHK(P.p_rtab.ensure(nr), "pre alloc");
        std::memcpy(P.p_rtab.p, P.rtab.data(), sizeof(double) * nr);
        PCHK(kcopy(P.d_rtab.p, P.p_rtab.p, sizeof(double) * nr, st), "pre H2D ranks");
        PCHK(kfill(P.fbad.p, 0, sizeof(int), st), "pre memset");
        bpk::k_pre_check<<<(n + B - 1) / B, B, 0, st>>>(d_lasers, n, P.d_rtab.p, nr, P.colflag.p, P.vrank.p, P.fbad.p);
        PCHK(kcopy(P.p_fbad.p, P.fbad.p, sizeof(int), st), "pre D2H check");
        PCHK(hipStreamSynchronize(st), "pre sync check");
        fast = P.p_fbad.p[0] == 0;
    }
    if (fast) {
        P.fast_runs++;
        PCHK(P.fkey.ensure(n2), "pre alloc"); PCHK(P.fkey2.ensure(n2), "pre alloc");
        tb = P.tmp.cap;
        PCHK(rocprim::inclusive_scan(P.tmp.p, tb, P.colflag.p, P.colid.p, (size_t)n, rocprim::plus<int>(), st),
             "pre scan columns");
        bpk::k_pre_fkeys<<<G, B, 0, st>>>(P.colid.p, P.vrank.p, P.vinit_rank, n2, P.fkey.p, P.val.p);
        const int bits = 9 + (32 - __builtin_clz((unsigned)n));  // column ids < n
        tb = P.tmp.cap;
        PCHK(rocprim::radix_sort_pairs(P.tmp.p, tb, P.fkey.p, P.fkey2.p, P.val.p, P.perm.p, (unsigned)n2, 0,
                                       std::min(bits, 32), st),
             "pre sort (column, vertical)");
    } else {
        P.general_runs++;
        bpk::k_pre_vkeys<<<G, B, 0, st>>>(d_lasers, n2, pp.vert_init, P.vkey.p, P.val.p);
        tb = P.tmp.cap;
        PCHK(rocprim::radix_sort_pairs(P.tmp.p, tb, P.vkey.p, P.vkey2.p, P.val.p, P.val2.p, (unsigned)n2, 0, 64, st),
             "pre sort vertical");
        bpk::k_pre_akeys<<<G, B, 0, st>>>(d_lasers, P.val2.p, n2, P.akey.p);
        tb = P.tmp.cap;
        PCHK(rocprim::radix_sort_pairs(P.tmp.p, tb, P.akey.p, P.akey2.p, P.val2.p, P.perm.p, (unsigned)n2, 0, 64, st),
             "pre sort azimuth");
    }
    bpk::k_pre_flags<<<G, B, 0, st>>>(d_lasers, P.perm.p, n2, pp.vert_init, P.cnt.p);
    tb = P.tmp.cap;
    PCHK(rocprim::inclusive_scan(P.tmp.p, tb, P.cnt.p, P.scan.p, (size_t)n2, rocprim::plus<unsigned long long>(), st),
         "pre scan cells");
    bpk::k_pre_starts<<<G, B, 0, st>>>(P.cnt.p, P.scan.p, n2, P.cstart.p, P.colcell.p, P.tot.p);
    bpk::k_pre_cells<<<G, B, 0, st>>>(d_lasers, P.perm.p, P.scan.p, P.cstart.p, selm, P.tot.p, pp.vert_init,
                                      P.syn_dist, n2, P.c_vr.p, P.c_dist.p, P.c_rm.p, P.c_sel.p, P.c_col.p,
                                      P.colmin.p);
    bpk::k_pre_colaz<<<G, B, 0, st>>>(d_lasers, P.colmin.p, P.tot.p, n2, P.col_az.p);
    bpk::k_pre_pts<<<G, B, 0, st>>>(P.c_vr.p, P.c_dist.p, P.c_col.p, P.col_az.p, P.tot.p, n2, P.pts.p);
    if (J > 0) PCHK(kfill(P.ph0.p, 0, sizeof(int) * J, st), "pre memset");
    c->stage_end(sg, st);
    PCHK(hipGetLastError(), "pre read launch");
    return BSHOT_OK;
}

// removeGround (src/preprocess.cpp:72-164)
int pre_ground(bshot_ctx* c) {
    PreState& P = pre_state(c);
    if (P.n <= 0) return BSHOT_OK;
    const int n2 = 2 * P.n, B = 256, G = (n2 + B - 1) / B;
    const int sg = c->stage_begin(BSHOT_STAGE_PRE, c->stream);
    bpk::k_pre_ground<<<G, B, 0, c->stream>>>(P.colcell.p, P.tot.p, n2, P.K, P.c_dist.p, P.pts.p, P.col_az.p,
                                              P.c_rm.p);
    c->stage_end(sg, c->stream);
    PCHK(hipGetLastError(), "pre ground launch");
    return BSHOT_OK;
}

// removeOccluded (src/preprocess.cpp:166-195)
int pre_occluded(bshot_ctx* c) {
    PreState& P = pre_state(c);
    const int J = (int)P.vj.size();
    if (P.n <= 0 || J == 0) return BSHOT_OK;
    const int n2 = 2 * P.n, B = 256, G = (n2 + B - 1) / B;
    // the column count is only known on the device: the table is sized for the worst case (one
    // column per event) and cleared on the device for the columns that exist
    PCHK(P.tab.ensure((size_t)n2 * J), "pre alloc table");
    hipStream_t st = c->stream;
    const int sg = c->stage_begin(BSHOT_STAGE_PRE, st);
    bpk::k_pre_tab_clear<<<1024, 256, 0, st>>>(P.tab.p, P.tot.p, J);
    bpk::k_pre_table<<<G, B, 0, st>>>(P.c_vr.p, P.c_col.p, P.tot.p, n2, P.d_vj.p, J, P.tab.p);
    bpk::k_pre_occl<<<J, 256, 0, st>>>(P.tab.p, J, P.tot.p, P.c_dist.p, P.col_az.p, P.K, P.c_rm.p, P.ph0.p);
    c->stage_end(sg, st);
    PCHK(hipGetLastError(), "pre occlusion launch");
    return BSHOT_OK;
}

// writePointCloud (src/preprocess.cpp:197-215): kept points -> d_xyz (float3 AoS, map order);
// syncs the stream for the count
int pre_write(bshot_ctx* c, float* d_xyz, int cap, int* n_out) {
    PreState& P = pre_state(c);
    if (P.n <= 0) {
        if (n_out) *n_out = 0;
        return BSHOT_OK;
    }
    const int n2 = 2 * P.n, B = 256, G = (n2 + B - 1) / B;
    hipStream_t st = c->stream;
    const int sg = c->stage_begin(BSHOT_STAGE_PRE, st);
    bpk::k_pre_keep<<<G, B, 0, st>>>(P.c_vr.p, P.c_dist.p, P.c_rm.p, P.c_sel.p, P.tot.p, n2, P.prm.vert_init,
                                     P.prm.save_sel ? 1 : 0, P.keep.p);
    size_t tb = P.tmp.cap;
    PCHK(rocprim::exclusive_scan(P.tmp.p, tb, P.keep.p, P.offs.p, 0, (size_t)n2, rocprim::plus<int>(), st),
         "pre scan keep");
    bpk::k_pre_write<<<G, B, 0, st>>>(P.pts.p, P.keep.p, P.offs.p, P.tot.p, n2, cap, d_xyz, P.tot.p + 2);
    c->stage_end(sg, st);
    PCHK(hipGetLastError(), "pre write launch");
    PCHK(kcopy(P.p_tot.p, P.tot.p, sizeof(int) * 4, st), "pre D2H count");
    PCHK(hipStreamSynchronize(st), "pre sync");
    c->resolve_events();
    P.cells = P.p_tot.p[0];
    P.cols = P.p_tot.p[1];
    P.counts_ok = true;
    if (n_out) *n_out = P.p_tot.p[2];
    if (P.p_tot.p[2] > cap)
        return c->fail("preprocess: output capacity " + std::to_string(cap) + " < " + std::to_string(P.p_tot.p[2]) +
                           " points",
                       BSHOT_ECAP);
    return BSHOT_OK;
}

int pre_run(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
            const bshot_pre_params* prm, const int32_t* sel, int nsel, float* d_xyz, int cap, int* n_out) {
    int rc;
    if ((rc = pre_read(c, d_lasers, n, vert_deg, nv, prm, sel, nsel))) return rc;
    if ((rc = pre_ground(c))) return rc;
    if ((rc = pre_occluded(c))) return rc;
    return pre_write(c, d_xyz, cap, n_out);
}

float* pre_out_buffer(bshot_ctx* c, int n) {
    PreState& P = pre_state(c);
    if (P.out.ensure(3 * (size_t)(n > 0 ? n : 1)) != hipSuccess) return nullptr;
    return P.out.p;
}

// rimg / rmmap / selmap of the last run as the reference's getters return them (include/preprocess.h:
// 36-38), merged into one table over rimg's keys in map order. Besides the cells, rimg holds the
// zero entries removeOccluded's operator[] reads insert (src/preprocess.cpp:177-178): at every
// vertical angle, in every column after the first, and in the first column when a later column has
// a non-zero range there; rmmap holds a 3 at such a first-column entry when the kernel flagged one.
int pre_cells(bshot_ctx* c, std::vector<bshot_pre_cell>& out) {
    out.clear();
    if (!c->prep) return BSHOT_OK;
    PreState& P = *c->prep;
    if (!P.counts_ok) {
        PCHK(kcopy(P.p_tot.p, P.tot.p, sizeof(int) * 4, c->stream), "pre D2H count");
        PCHK(hipStreamSynchronize(c->stream), "pre sync");
        P.cells = P.p_tot.p[0];
        P.cols = P.p_tot.p[1];
        P.counts_ok = true;
    }
    PCHK(hipStreamSynchronize(c->stream), "pre sync");
    const int M = P.cells, C = P.cols, J = (int)P.vj.size();
    std::vector<double> vr(M), dist(M), az(C);
    std::vector<int> rm(M), sl(M), col(M), ph0(J > 0 ? J : 1, 0);
    if (M > 0) {
        PCHK(hipMemcpy(vr.data(), P.c_vr.p, sizeof(double) * M, hipMemcpyDeviceToHost), "pre D2H cells");
        PCHK(hipMemcpy(dist.data(), P.c_dist.p, sizeof(double) * M, hipMemcpyDeviceToHost), "pre D2H cells");
        PCHK(hipMemcpy(rm.data(), P.c_rm.p, sizeof(int) * M, hipMemcpyDeviceToHost), "pre D2H cells");
        PCHK(hipMemcpy(sl.data(), P.c_sel.p, sizeof(int) * M, hipMemcpyDeviceToHost), "pre D2H cells");
        PCHK(hipMemcpy(col.data(), P.c_col.p, sizeof(int) * M, hipMemcpyDeviceToHost), "pre D2H cells");
        PCHK(hipMemcpy(az.data(), P.col_az.p, sizeof(double) * C, hipMemcpyDeviceToHost), "pre D2H cells");
        if (J > 0) PCHK(hipMemcpy(ph0.data(), P.ph0.p, sizeof(int) * J, hipMemcpyDeviceToHost), "pre D2H cells");
    }
    // per column, its entries keyed by vertical (std::map: the reference's inner-map order)
    std::vector<std::map<double, bshot_pre_cell>> cols((size_t)C);
    for (int m = 0; m < M; ++m) cols[col[m]][vr[m]] = bshot_pre_cell{az[col[m]], vr[m], dist[m], rm[m], sl[m]};
    for (int j = 0; j < J; ++j) {
        const double v = P.vj[j];
        bool later_nonzero = false;
        for (int cc = 1; cc < C; ++cc) {
            auto it = cols[cc].find(v);
            if (it == cols[cc].end()) cols[cc][v] = bshot_pre_cell{az[cc], v, 0.0, -1, -1};
            else if (it->second.distance != 0) later_nonzero = true;
        }
        if (C > 0 && later_nonzero && cols[0].find(v) == cols[0].end())
            cols[0][v] = bshot_pre_cell{az[0], v, 0.0, ph0[j] ? 3 : -1, -1};
    }
    for (int cc = 0; cc < C; ++cc)
        for (auto& kv : cols[cc]) out.push_back(kv.second);
    return BSHOT_OK;
}

}  // namespace bsh

extern "C" {

void bshot_pre_default_params(bshot_pre_params* p) {
    p->vert_init = -0.6;   // src/preprocess.cpp:7
    p->lowpt_th = -2000;   // include/preprocess.h:43
    p->have_sel_list = 0;  // src/preprocess.cpp:5
    p->save_sel = 1;       // src/preprocess.cpp:6
}

int bshot_preprocess_device(bshot_ctx* c, const bshot_laser* d_lasers, int n, const double* vert_deg, int nv,
                            const bshot_pre_params* prm, const int32_t* sel, int nsel, float* d_xyz, int cap,
                            int* n_out) {
    if (!c || n < 0 || (n > 0 && !d_lasers) || nv < 0 || (nv > 0 && !vert_deg) || cap < 0 ||
        (cap > 0 && !d_xyz) || n > (1 << 28))
        return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    return bsh::pre_run(c, d_lasers, n, vert_deg, nv, prm, sel, nsel, d_xyz, cap, n_out);
}

int bshot_preprocess(bshot_ctx* c, const bshot_laser* lasers, int n, const double* vert_deg, int nv,
                     const bshot_pre_params* prm, const int32_t* sel, int nsel, float* xyz, int cap, int* n_out) {
    if (!c || n < 0 || (n > 0 && !lasers) || nv < 0 || (nv > 0 && !vert_deg) || cap < 0 || (cap > 0 && !xyz) ||
        n > (1 << 28))
        return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    const bshot_laser* d = nullptr;
    int rc = bsh::pre_stage_lasers(c, lasers, n, &d);
    if (rc) return rc;
    float* out = bsh::pre_out_buffer(c, n);  // at most one point per laser
    if (!out) return c->fail("pre alloc out", BSHOT_EHIP);
    int np = 0;
    if ((rc = bsh::pre_run(c, d, n, vert_deg, nv, prm, sel, nsel, out, n, &np))) return rc;
    if (n_out) *n_out = np;
    if (np > cap) return c->fail("preprocess: output capacity too small", BSHOT_ECAP);
    if (np > 0 && hipMemcpy(xyz, out, sizeof(float) * 3 * (size_t)np, hipMemcpyDeviceToHost) != hipSuccess)
        return c->fail("pre D2H points", BSHOT_EHIP);
    return BSHOT_OK;
}

int bshot_preprocess_cells(bshot_ctx* c, bshot_pre_cell* out, int cap, int* n_out) {
    if (!c || cap < 0 || (cap > 0 && !out)) return BSHOT_EINVAL;
    (void)hipSetDevice(c->device);
    std::vector<bshot_pre_cell> v;
    const int rc = bsh::pre_cells(c, v);
    if (rc) return rc;
    const int k = (int)v.size();
    if (n_out) *n_out = k;
    if (k > cap) return BSHOT_ECAP;
    if (k > 0) std::memcpy(out, v.data(), sizeof(bshot_pre_cell) * (size_t)k);
    return BSHOT_OK;
}

}  // extern "C"
