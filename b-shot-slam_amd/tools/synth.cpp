// synth.cpp -- deterministic synthetic Velodyne sweeps. Input generator for
// tests and bench.py (the reference ships no data: .gitignore:4 ignores data/*). Not on the hot path.
//
// Scene (world frame, mm): ground z=-1730; facade rows at x=+-9000 in segments separated by cross
// streets, with recessed windows (300 mm) and doors (500 mm); a back row of buildings at
// x=+-35000; poles r=150 every 12 m at x=+-7000; parked cars (1800x4500x1500 boxes) at x=+-3600;
// trees (spheres r~1500) at x=+-6000. Scene seeds with bit 31 set select an aperiodic variant
// (diagnostic, tests/diag/config3_diag.py): pole spacing 6-18 m instead of 12 m, and each 4 m
// facade cell draws its own window presence, width and height from a hash. Sensor pose at frame t: yaw_t = 0.5deg*sin(2*pi*t/200),
// position (0, 800*t, 0). Returns: nearest hit, range < max_range, range noise N(0, 20 mm)
// quantised to 2 mm (src/preprocess.cpp:45-46 uses 2 mm ticks). Output order: azimuth-major,
// vertical-ascending (mimics src/preprocess.cpp:201-215). Points are in the sensor frame.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace {

struct Prim {
    int kind;  // 0 facade segment, 1 pole (vertical cylinder), 2 box, 3 sphere, 4 back plane segment
    double a[8];
    double ymin, ymax;
};

static inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline double u01(uint64_t h) { return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

struct Scene {
    std::vector<Prim> prims;  // sorted by ymin
    bool aperiodic = false;
    explicit Scene(uint32_t seed) {
        aperiodic = (seed & 0x80000000u) != 0;
        uint64_t st = seed * 0x1234567ull + 99;
        auto rnd = [&]() { st = splitmix(st); return u01(st); };
        const double Y0 = -200000, Y1 = 1300000;
        for (int side = -1; side <= 1; side += 2) {
            // facade segments with cross streets
            double y = Y0;
            while (y < Y1) {
                const double len = 20000 + 40000 * rnd();
                const double h = 6000 + 9000 * rnd();
                Prim p{};
                p.kind = 0;
                p.a[0] = side * 9000.0; p.a[1] = y; p.a[2] = y + len; p.a[3] = -1730 + h; p.a[4] = side;
                p.a[5] = 4000 * rnd();  // window phase
                p.a[6] = (double)(splitmix(st) >> 12);  // per-facade salt of the aperiodic variant
                p.ymin = y; p.ymax = y + len;
                prims.push_back(p);
                y += len + 12000 + 8000 * rnd();
            }
            Prim bp{};
            bp.kind = 4;
            bp.a[0] = side * 35000.0; bp.a[3] = -1730 + 20000;
            bp.ymin = Y0 - 200000; bp.ymax = Y1 + 200000;
            prims.push_back(bp);
            for (double py = Y0 + 3000 * (side + 2); py < Y1; py += aperiodic ? 6000 + 12000 * rnd() : 12000) {
                Prim p{};
                p.kind = 1;
                p.a[0] = side * 7000.0; p.a[1] = py; p.a[2] = 150; p.a[3] = -1730; p.a[4] = 3270;
                p.ymin = py - 150; p.ymax = py + 150;
                prims.push_back(p);
                Prim t{};
                t.kind = 3;
                const double r = 1200 + 600 * rnd();
                t.a[0] = side * 6000.0; t.a[1] = py + 6000; t.a[2] = 2300 + 800 * rnd(); t.a[3] = r;
                t.ymin = t.a[1] - r; t.ymax = t.a[1] + r;
                if (rnd() < 0.7) prims.push_back(t);
            }
            for (double cy = Y0; cy < Y1; cy += 7000 + 6000 * rnd()) {
                if (rnd() < 0.45) continue;
                Prim b{};
                b.kind = 2;
                const double cx = side * (3600 + 300 * rnd());
                b.a[0] = cx - 900; b.a[1] = cx + 900; b.a[2] = cy; b.a[3] = cy + 4500; b.a[4] = -1730; b.a[5] = -1730 + 1400 + 200 * rnd();
                b.ymin = cy; b.ymax = cy + 4500;
                prims.push_back(b);
            }
        }
        std::sort(prims.begin(), prims.end(), [](const Prim& l, const Prim& r) { return l.ymin < r.ymin; });
    }
};

static std::mutex g_mu;
static std::map<uint32_t, std::shared_ptr<Scene>> g_scenes;
static std::shared_ptr<Scene> get_scene(uint32_t seed) {
    std::lock_guard<std::mutex> l(g_mu);
    auto it = g_scenes.find(seed);
    if (it != g_scenes.end()) return it->second;
    auto s = std::make_shared<Scene>(seed);
    g_scenes[seed] = s;
    return s;
}

// nearest positive ray parameter of one primitive (inf if none); ray o + t d, |d| = 1
static double hit(const Prim& p, const double o[3], const double d[3], bool& is_ground, bool aperiodic) {
    const double INF = 1e300;
    is_ground = false;
    switch (p.kind) {
        case 0: {  // facade plane x = X facing the street, window/door recesses
            if (std::fabs(d[0]) < 1e-12) return INF;
            const double X = p.a[0];
            double t = (X - o[0]) / d[0];
            if (t <= 0) return INF;
            double y = o[1] + t * d[1], z = o[2] + t * d[2];
            if (y < p.a[1] || y > p.a[2] || z < -1730 || z > p.a[3]) return INF;
            const double u = std::fmod(y - p.a[1] + p.a[5], 4000.0);
            const double fz = z + 1730;
            double recess = 0;
            if (aperiodic) {
                // every 4 m x 3.5 m facade cell draws its window (present, x-extent, height) from a hash
                const int64_t cx = (int64_t)std::floor((y - p.a[1] + p.a[5]) / 4000.0);
                const int64_t cz = fz > 1000 ? (int64_t)std::floor((fz - 1000) / 3500.0) : -1;
                const uint64_t hw = splitmix((uint64_t)p.a[6] ^ ((uint64_t)cx << 8) ^ (uint64_t)(cz + 1));
                const double w0 = 300 + 1500 * u01(hw), w1 = w0 + 700 + 1300 * u01(splitmix(hw + 1));
                const double hh = 1000 + 1500 * u01(splitmix(hw + 2));
                if (cz >= 0 && (hw & 7) < 5 && std::fmod(fz - 1000, 3500.0) < hh && u > w0 && u < w1 &&
                    fz < p.a[3] + 1730 - 800)
                    recess = 300;
                if (fz < 2200 && u > 200 && u < 1400 && (splitmix(hw + 3) & 3) == 0) recess = 500;
            } else {
            if (fz > 1000 && std::fmod(fz - 1000, 3500.0) < 1800 && u > 1200 && u < 2700 && fz < p.a[3] + 1730 - 800) recess = 300;
            if (fz < 2200 && u > 200 && u < 1400 && std::fmod(y - p.a[1], 12000.0) < 4000) recess = 500;
            }
            if (recess > 0) {
                const double t2 = (X + p.a[4] * recess - o[0]) / d[0];
                if (t2 > 0) return t2;
            }
            return t;
        }
        case 4: {
            if (std::fabs(d[0]) < 1e-12) return INF;
            const double t = (p.a[0] - o[0]) / d[0];
            if (t <= 0) return INF;
            const double z = o[2] + t * d[2];
            if (z < -1730 || z > p.a[3]) return INF;
            return t;
        }
        case 1: {  // vertical cylinder
            const double ox = o[0] - p.a[0], oy = o[1] - p.a[1];
            const double A = d[0] * d[0] + d[1] * d[1];
            if (A < 1e-18) return INF;
            const double B = 2 * (ox * d[0] + oy * d[1]);
            const double C = ox * ox + oy * oy - p.a[2] * p.a[2];
            const double disc = B * B - 4 * A * C;
            if (disc < 0) return INF;
            const double t = (-B - std::sqrt(disc)) / (2 * A);
            if (t <= 0) return INF;
            const double z = o[2] + t * d[2];
            if (z < p.a[3] || z > p.a[4]) return INF;
            return t;
        }
        case 2: {  // axis-aligned box, slab test
            double t0 = 0, t1 = 1e300;
            const double lo[3] = {p.a[0], p.a[2], p.a[4]}, hi[3] = {p.a[1], p.a[3], p.a[5]};
            for (int k = 0; k < 3; ++k) {
                if (std::fabs(d[k]) < 1e-15) {
                    if (o[k] < lo[k] || o[k] > hi[k]) return INF;
                    continue;
                }
                double ta = (lo[k] - o[k]) / d[k], tb = (hi[k] - o[k]) / d[k];
                if (ta > tb) std::swap(ta, tb);
                t0 = std::max(t0, ta);
                t1 = std::min(t1, tb);
                if (t0 > t1) return INF;
            }
            return t0 > 0 ? t0 : INF;
        }
        case 3: {  // sphere
            const double ox = o[0] - p.a[0], oy = o[1] - p.a[1], oz = o[2] - p.a[2];
            const double B = ox * d[0] + oy * d[1] + oz * d[2];
            const double C = ox * ox + oy * oy + oz * oz - p.a[3] * p.a[3];
            const double disc = B * B - C;
            if (disc < 0) return INF;
            const double t = -B - std::sqrt(disc);
            return t > 0 ? t : INF;
        }
    }
    return INF;
}

}  // namespace

extern "C" {

// sensor: 0 = HDL-64 (64 x 2048), 1 = VLP-128 style (128 x 2000). Returns the point count
// (or -needed when cap is too small). pose_out (nullable): row-major 4x4 sensor->world pose.
int synth_sweep(int sensor, uint32_t scene_seed, int frame, int no_ground, float max_range, float* xyz, int cap,
                float* pose_out) {
    auto sc = get_scene(scene_seed);
    std::vector<double> beams;
    int A;
    if (sensor == 0) {
        A = 2048;
        for (int i = 0; i < 32; ++i) beams.push_back(2.0 + (-8.33 - 2.0) * i / 31.0);
        for (int i = 0; i < 32; ++i) beams.push_back(-8.83 + (-24.33 + 8.83) * i / 31.0);
    } else {
        A = 2000;
        for (int i = 0; i < 128; ++i) beams.push_back(-25.0 + 40.0 * i / 127.0);
    }
    std::sort(beams.begin(), beams.end());
    const int V = (int)beams.size();
    const double yaw = 0.5 * M_PI / 180.0 * std::sin(2 * M_PI * frame / 200.0);
    const double cy = std::cos(yaw), sy = std::sin(yaw);
    const double o[3] = {0.0, 800.0 * frame, 0.0};
    if (pose_out) {
        const float P[16] = {(float)cy, (float)-sy, 0, (float)o[0], (float)sy, (float)cy, 0, (float)o[1],
                             0, 0, 1, (float)o[2], 0, 0, 0, 1};
        std::memcpy(pose_out, P, sizeof(P));
    }
    // candidate primitives near the sensor
    std::vector<const Prim*> near;
    for (const Prim& p : sc->prims)
        if (p.ymax >= o[1] - max_range - 1000 && p.ymin <= o[1] + max_range + 1000) near.push_back(&p);
    std::vector<float> out((size_t)A * V * 3);
    std::vector<uint8_t> valid((size_t)A * V, 0);
#pragma omp parallel for schedule(static)
    for (int j = 0; j < A; ++j) {
        const double az = 2 * M_PI * j / A;
        for (int b = 0; b < V; ++b) {
            const double v = beams[b] * M_PI / 180.0;
            const double ds[3] = {std::cos(v) * std::sin(az), std::cos(v) * std::cos(az), std::sin(v)};
            const double d[3] = {cy * ds[0] - sy * ds[1], sy * ds[0] + cy * ds[1], ds[2]};
            double best = 1e300;
            bool ground = false;
            if (d[2] < -1e-12) {
                best = (-1730.0 - o[2]) / d[2];
                ground = true;
            }
            for (const Prim* p : near) {
                bool g;
                const double t = hit(*p, o, d, g, sc->aperiodic);
                if (t < best) { best = t; ground = false; }
            }
            if (best >= 1e299 || (no_ground && ground)) continue;
            const uint64_t h = splitmix(((uint64_t)scene_seed << 40) ^ ((uint64_t)(frame + 1000) << 20) ^ (uint64_t)(j * V + b));
            const double u1 = u01(h), u2 = u01(splitmix(h));
            const double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(2 * M_PI * u2);
            const double r = std::round((best + 20.0 * g) / 2.0) * 2.0;
            if (!(r < max_range) || r <= 0) continue;
            const size_t id = (size_t)j * V + b;
            out[3 * id] = (float)(r * ds[0]);
            out[3 * id + 1] = (float)(r * ds[1]);
            out[3 * id + 2] = (float)(r * ds[2]);
            valid[id] = 1;
        }
    }
    int n = 0;
    for (size_t id = 0; id < valid.size(); ++id) n += valid[id];
    if (n > cap) return -n;
    int m = 0;
    for (size_t id = 0; id < valid.size(); ++id)
        if (valid[id]) { std::memcpy(xyz + 3 * (size_t)m, &out[3 * id], 12); ++m; }
    return n;
}

// Velodyne laser returns of one rotation (velodyne::Laser records, include/VelodyneCapture.h:43-50,
// 32 B: azimuth deg, vertical deg, distance in 2 mm units, intensity, id, time) -- the input of the
// preprocessor (src/preprocess.cpp:38-70). sensor: 0 HDL-64 (64 x 2048), 1 VLP-128 style
// (128 x 2000), 2 HDL-32E (32 x 2170, the capture's vertical table, include/VelodyneCapture.h:572).
// Records come in firing order (azimuth-major, laser id inside a firing), azimuth in the packet's
// 0.01 deg steps; a return beyond max_range or without a hit is distance 0 (a lost point, as the
// sensor reports it). The sensor sits sensor_height mm above the ground plane. Returns the record
// count (or -needed when cap is too small).
struct SynthLaser {
    double azimuth;
    double vertical;
    uint16_t distance;
    uint8_t intensity;
    uint8_t id;
    int64_t time;
};
static_assert(sizeof(SynthLaser) == 32, "velodyne::Laser layout");

int synth_lasers(int sensor, uint32_t scene_seed, int frame, float max_range, float sensor_height, void* out_v,
                 int cap) {
    SynthLaser* out = static_cast<SynthLaser*>(out_v);
    auto sc = get_scene(scene_seed);
    std::vector<double> beams;
    int A;
    if (sensor == 0) {
        A = 2048;
        for (int i = 0; i < 32; ++i) beams.push_back(2.0 + (-8.33 - 2.0) * i / 31.0);
        for (int i = 0; i < 32; ++i) beams.push_back(-8.83 + (-24.33 + 8.83) * i / 31.0);
    } else if (sensor == 1) {
        A = 2000;
        for (int i = 0; i < 128; ++i) beams.push_back(-25.0 + 40.0 * i / 127.0);
    } else {
        A = 2170;
        beams = {-30.67, -9.3299999, -29.33, -8.0, -28, -6.6700001, -26.67, -5.3299999, -25.33, -4.0, -24.0,
                 -2.6700001, -22.67, -1.33, -21.33, 0.0, -20.0, 1.33, -18.67, 2.6700001, -17.33, 4.0, -16,
                 5.3299999, -14.67, 6.6700001, -13.33, 8.0, -12.0, 9.3299999, -10.67, 10.67};
    }
    const int V = (int)beams.size();
    if ((long long)A * V > cap) return -(A * V);
    const double yaw = 0.5 * M_PI / 180.0 * std::sin(2 * M_PI * frame / 200.0);
    const double cy = std::cos(yaw), sy = std::sin(yaw);
    const double o[3] = {0.0, 800.0 * frame, sensor_height - 1730.0};
    std::vector<const Prim*> near;
    for (const Prim& p : sc->prims)
        if (p.ymax >= o[1] - max_range - 1000 && p.ymin <= o[1] + max_range + 1000) near.push_back(&p);
#pragma omp parallel for schedule(static)
    for (int j = 0; j < A; ++j) {
        const int rot = (int)std::lround(36000.0 * j / A) % 36000;  // rotational position, 0.01 deg
        const double az_deg = rot / 100.0;
        const double az = az_deg * M_PI / 180.0;
        for (int b = 0; b < V; ++b) {
            const double v = beams[b] * M_PI / 180.0;
            const double ds[3] = {std::cos(v) * std::sin(az), std::cos(v) * std::cos(az), std::sin(v)};
            const double d[3] = {cy * ds[0] - sy * ds[1], sy * ds[0] + cy * ds[1], ds[2]};
            double best = 1e300;
            if (d[2] < -1e-12) best = (-1730.0 - o[2]) / d[2];
            for (const Prim* p : near) {
                bool g;
                const double t = hit(*p, o, d, g, sc->aperiodic);
                if (t < best) best = t;
            }
            const uint64_t h = splitmix(((uint64_t)scene_seed << 40) ^ ((uint64_t)(frame + 1000) << 20) ^ (uint64_t)(j * V + b));
            const double u1 = u01(h), u2 = u01(splitmix(h));
            const double g = std::sqrt(-2.0 * std::log(u1)) * std::cos(2 * M_PI * u2);
            double r = best >= 1e299 ? 0.0 : std::round((best + 20.0 * g) / 2.0) * 2.0;
            if (!(r < max_range) || r <= 0) r = 0;
            SynthLaser& L = out[(size_t)j * V + b];
            L.azimuth = az_deg;
            L.vertical = beams[b];
            L.distance = (uint16_t)(r / 2);
            L.intensity = (uint8_t)(splitmix(h) & 0xFF);
            L.id = (uint8_t)b;
            L.time = frame;
        }
    }
    return A * V;
}

}  // extern "C"
