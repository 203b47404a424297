// pbstream ingest: the submaps and node clouds a ConstraintBuilder2D reads,
// straight out of a serialized state file, with no protobuf runtime.
//
// Stream framing follows io/proto_stream.cc:26-43 and :68-86 (an 8-byte
// little-endian magic, then per message an 8-byte little-endian size and a
// gzip member). The first message is a SerializationHeader
// (mapping/proto/serialization.proto:72-74); every later one is a
// SerializedData whose oneof we keep for `submap` (3) and `node` (4)
// (serialization.proto:76-88); everything else is skipped by wire type.
// Field numbers: Submap :26-30, Node :32-35, Submap2D (submap.proto:24-29),
// Grid2D (grid_2d.proto:22-42), MapLimits (map_limits.proto:22-26),
// CellLimits (cell_limits_2d.proto:19-22), TrajectoryNodeData
// (trajectory_node_data.proto:23-32), CompressedPointCloud
// (sensor/proto/sensor.proto:33-36), Rigid3d / Vector / Quaterniond
// (transform/proto/transform.proto).
//
// Grid values follow Grid2D::Grid2D(proto) (mapping/2d/grid_2d.cc:75-96): the
// 0/0 correspondence-cost pair of older files loads as kMin/kMaxCorrespondence
// Cost (:22-44), cells must fit uint16 (:93). Clouds decode exactly as
// CompressedPointCloud::ConstIterator (sensor/compressed_point_cloud.cc:79-97):
// int block origin + raster offset, times 0.001f.
//
// 3D: Submap3D (submap.proto:32-39) keeps both HybridGrids (hybrid_grid.proto:
// resolution, sint32 x/y/z indices, int32 values) and the rotational
// histogram; values load as HybridGrid(proto) (mapping/3d/hybrid_grid.h:
// 473-484) does, through ValueToProbability then ProbabilityToValue
// (probability_values.cc:27-49, probability_values.h:32-93), so an unknown 0
// loads as 1 and the update marker is dropped. Nodes also keep their high /
// low resolution clouds and histogram (trajectory_node_data.proto:28-30).
#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/csm_amd.h"

namespace {

constexpr uint64_t kMagic = 0x7b1d1f7b5bf501dbull;  // proto_stream.cc:27

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  bool Done() const { return !ok || p >= end; }
  uint64_t Varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) {
        ok = false;
        return 0;
      }
      const uint8_t b = *p++;
      v |= static_cast<uint64_t>(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  uint64_t Fixed(int bytes) {
    if (end - p < bytes) {
      ok = false;
      p = end;
      return 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < bytes; ++i) v |= static_cast<uint64_t>(p[i]) << (8 * i);
    p += bytes;
    return v;
  }
  Reader Sub() {
    const uint64_t n = Varint();
    if (!ok || n > static_cast<uint64_t>(end - p)) {
      ok = false;
      p = end;
      return Reader{end, end, false};
    }
    Reader r{p, p + n};
    p += n;
    return r;
  }
  void Skip(int wire) {
    switch (wire) {
      case 0: Varint(); break;
      case 1: Fixed(8); break;
      case 2: Sub(); break;
      case 5: Fixed(4); break;
      default: ok = false; p = end;
    }
  }
  double Double(int wire) {
    if (wire != 1) {
      Skip(wire);
      return 0.;
    }
    const uint64_t bits = Fixed(8);
    double d;
    std::memcpy(&d, &bits, 8);
    return d;
  }
  float Float(int wire) {
    if (wire != 5) {
      Skip(wire);
      return 0.f;
    }
    const uint32_t bits = static_cast<uint32_t>(Fixed(4));
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
  }
  int64_t Int(int wire) {
    if (wire != 0) {
      Skip(wire);
      return 0;
    }
    return static_cast<int64_t>(Varint());
  }
};

// Calls fn(field, wire, reader) for every field of the message in r; fn reads
// or skips the value. Returns false on malformed input.
template <class Fn>
bool Fields(Reader r, Fn fn) {
  while (!r.Done()) {
    const uint64_t key = r.Varint();
    if (!r.ok) break;
    const int field = static_cast<int>(key >> 3), wire = static_cast<int>(key & 7);
    if (field == 0) return false;
    fn(field, wire, r);
  }
  return r.ok;
}

// repeated int32, packed (proto3 default) or one value per key.
void Int32s(int wire, Reader& r, std::vector<int32_t>* out) {
  if (wire == 2) {
    Reader s = r.Sub();
    while (!s.Done()) out->push_back(static_cast<int32_t>(s.Varint()));
    if (!s.ok) r.ok = false;
  } else if (wire == 0) {
    out->push_back(static_cast<int32_t>(r.Varint()));
  } else {
    r.Skip(wire);
  }
}

// repeated sint32 (zigzag), packed or not.
void SInt32s(int wire, Reader& r, std::vector<int32_t>* out) {
  auto zz = [](uint64_t n) {
    const uint32_t u = static_cast<uint32_t>(n);
    return static_cast<int32_t>((u >> 1) ^ (~(u & 1) + 1));
  };
  if (wire == 2) {
    Reader s = r.Sub();
    while (!s.Done()) out->push_back(zz(s.Varint()));
    if (!s.ok) r.ok = false;
  } else if (wire == 0) {
    out->push_back(zz(r.Varint()));
  } else {
    r.Skip(wire);
  }
}

// repeated float, packed (fixed32 run) or one value per key.
void Floats(int wire, Reader& r, std::vector<float>* out) {
  if (wire == 2) {
    Reader s = r.Sub();
    while (!s.Done()) out->push_back(s.Float(5));
    if (!s.ok) r.ok = false;
  } else {
    out->push_back(r.Float(wire));
  }
}

bool Vec(Reader r, double* v, int n) {
  return Fields(r, [&](int f, int w, Reader& x) {
    if (f >= 1 && f <= n) v[f - 1] = x.Double(w);
    else x.Skip(w);
  });
}

// transform.proto Quaterniond is (x=1, y=2, z=3, w=4); we store (w, x, y, z).
bool Quat(Reader r, double* wxyz) {
  double xyzw[4] = {0., 0., 0., 0.};
  const bool ok = Vec(r, xyzw, 4);
  wxyz[0] = xyzw[3];
  wxyz[1] = xyzw[0];
  wxyz[2] = xyzw[1];
  wxyz[3] = xyzw[2];
  return ok;
}

// Rigid3d -> (tx, ty, tz, qw, qx, qy, qz).
bool Rigid(Reader r, double* pose7) {
  bool ok = true;
  ok &= Fields(r, [&](int f, int w, Reader& x) {
    if (f == 1 && w == 2) ok &= Vec(x.Sub(), pose7, 3);
    else if (f == 2 && w == 2) ok &= Quat(x.Sub(), pose7 + 3);
    else x.Skip(w);
  });
  return ok;
}

// Largest decompressed message accepted (a 400x400 Submap2D is ~0.5 MB, a
// 3D submap's two HybridGrids tens of MB). A stream whose message inflates
// past this is rejected rather than exhausting host memory.
// CSM_PBSTREAM_MAX_MESSAGE_BYTES lowers (or raises) the limit.
size_t MaxMessageBytes() {
  size_t limit = size_t{256} << 20;
  if (const char* e = std::getenv("CSM_PBSTREAM_MAX_MESSAGE_BYTES")) {
    const long long v = std::atoll(e);
    if (v > 0) limit = static_cast<size_t>(v);
  }
  return limit;
}

bool Gunzip(const std::vector<uint8_t>& in, std::string* out) {
  const size_t limit = MaxMessageBytes();
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return false;
  zs.next_in = const_cast<Bytef*>(in.data());
  zs.avail_in = static_cast<uInt>(in.size());
  out->clear();
  char buf[1 << 16];
  int rc;
  do {
    zs.next_out = reinterpret_cast<Bytef*>(buf);
    zs.avail_out = sizeof(buf);
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&zs);
      return false;
    }
    const size_t got = sizeof(buf) - zs.avail_out;
    if (out->size() + got > limit) {
      inflateEnd(&zs);
      return false;
    }
    out->append(buf, got);
  } while (rc != Z_STREAM_END);
  inflateEnd(&zs);
  return true;
}

struct Submap2DRec {
  int32_t trajectory_id = 0, submap_index = 0;
  csm_map_limits limits{};
  float min_cc = 0.f, max_cc = 0.f;
  int32_t finished = 0;
  double local_pose[7] = {0., 0., 0., 1., 0., 0., 0.};
  std::vector<uint16_t> cells;
};

struct NodeRec {
  int32_t trajectory_id = 0, node_index = 0;
  int64_t timestamp = 0;
  double local_pose[7] = {0., 0., 0., 1., 0., 0., 0.};
  double gravity_alignment[4] = {1., 0., 0., 0.};
  std::vector<float> clouds[3];  // filtered gravity-aligned, high, low resolution
  std::vector<float> histogram;
};

struct HybridGridRec {
  float resolution = 0.f;
  std::vector<int32_t> xyz;  // 3 per cell
  std::vector<uint16_t> values;
};

struct Submap3DRec {
  int32_t trajectory_id = 0, submap_index = 0;
  int32_t finished = 0;
  double local_pose[7] = {0., 0., 0., 1., 0., 0., 0.};
  HybridGridRec grids[2];  // high, low resolution
  std::vector<float> histogram;
};

// ProbabilityToValue(ValueToProbability(v)): PrecomputeValueToBoundedFloat's
// table (probability_values.cc:27-49, both update-marker halves) followed by
// BoundedFloatToValue (probability_values.h:32-45).
uint16_t LoadedProbabilityValue(uint16_t value) {
  const float kMinProbability = 0.1f, kMaxProbability = 1.f - kMinProbability;
  const uint16_t v = value & 0x7fff;
  float p = kMinProbability;
  if (v != 0) {
    const float kScale = (kMaxProbability - kMinProbability) / (32768 - 2.f);
    p = static_cast<float>(v) * kScale + (kMinProbability - kScale);
  }
  const float c = std::fmin(std::fmax(p, kMinProbability), kMaxProbability);
  return static_cast<uint16_t>(
      std::lround((c - kMinProbability) * (32766.f / (kMaxProbability - kMinProbability))) + 1);
}

int ParseHybridGrid(Reader r, HybridGridRec* g) {
  std::vector<int32_t> x, y, z, values;
  bool ok = Fields(r, [&](int f, int w, Reader& q) {
    if (f == 1) g->resolution = q.Float(w);
    else if (f == 3) SInt32s(w, q, &x);
    else if (f == 4) SInt32s(w, q, &y);
    else if (f == 5) SInt32s(w, q, &z);
    else if (f == 6) Int32s(w, q, &values);
    else q.Skip(w);
  });
  if (!ok || x.size() != values.size() || y.size() != values.size() ||
      z.size() != values.size())  // hybrid_grid.h:475-477
    return CSM_EINVAL;
  g->xyz.resize(3 * values.size());
  g->values.resize(values.size());
  for (size_t i = 0; i < values.size(); ++i) {
    if (values[i] < 0 || values[i] > 0xffff) return CSM_EINVAL;
    g->xyz[3 * i] = x[i];
    g->xyz[3 * i + 1] = y[i];
    g->xyz[3 * i + 2] = z[i];
    g->values[i] = LoadedProbabilityValue(static_cast<uint16_t>(values[i]));
  }
  return CSM_OK;
}

bool ParseLimits(Reader r, csm_map_limits* l) {
  bool ok = true;
  ok &= Fields(r, [&](int f, int w, Reader& x) {
    if (f == 1) {
      l->resolution = x.Double(w);
    } else if (f == 2 && w == 2) {
      double m[2] = {0., 0.};
      ok &= Vec(x.Sub(), m, 2);
      l->max_x = m[0];
      l->max_y = m[1];
    } else if (f == 3 && w == 2) {
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        if (g == 1) l->num_x_cells = static_cast<int32_t>(y.Int(v));
        else if (g == 2) l->num_y_cells = static_cast<int32_t>(y.Int(v));
        else y.Skip(v);
      });
    } else {
      x.Skip(w);
    }
  });
  return ok;
}

int ParseGrid(Reader r, Submap2DRec* s) {
  std::vector<int32_t> cells;
  bool ok = true;
  ok &= Fields(r, [&](int f, int w, Reader& x) {
    if (f == 1 && w == 2) ok &= ParseLimits(x.Sub(), &s->limits);
    else if (f == 2) Int32s(w, x, &cells);
    else if (f == 6) s->min_cc = x.Float(w);
    else if (f == 7) s->max_cc = x.Float(w);
    else x.Skip(w);
  });
  if (!ok) return CSM_EINVAL;
  if (s->min_cc == 0.f && s->max_cc == 0.f) {
    // kMinCorrespondenceCost / kMaxCorrespondenceCost (probability_values.h).
    const float kMinProbability = 0.1f, kMaxProbability = 1.f - kMinProbability;
    s->min_cc = 1.f - kMaxProbability;
    s->max_cc = 1.f - kMinProbability;
  }
  if (!(s->min_cc < s->max_cc)) return CSM_EINVAL;  // grid_2d.cc:84
  const int64_t n = static_cast<int64_t>(s->limits.num_x_cells) * s->limits.num_y_cells;
  if (s->limits.num_x_cells < 0 || s->limits.num_y_cells < 0 ||
      n != static_cast<int64_t>(cells.size()))
    return CSM_EINVAL;
  s->cells.resize(cells.size());
  for (size_t i = 0; i < cells.size(); ++i) {
    if (cells[i] < 0 || cells[i] > 0xffff) return CSM_EINVAL;  // grid_2d.cc:93
    s->cells[i] = static_cast<uint16_t>(cells[i]);
  }
  return CSM_OK;
}

// Returns 1 when a Submap2D was read into *s, 2 for a Submap3D read into *s3.
int ParseSubmap(Reader r, Submap2DRec* s, Submap3DRec* s3) {
  bool ok = true, is2d = false, is3d = false;
  int rc = CSM_OK;
  ok &= Fields(r, [&](int f, int w, Reader& x) {
    if (f == 1 && w == 2) {
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        if (g == 1) s->trajectory_id = s3->trajectory_id = static_cast<int32_t>(y.Int(v));
        else if (g == 2) s->submap_index = s3->submap_index = static_cast<int32_t>(y.Int(v));
        else y.Skip(v);
      });
    } else if (f == 3 && w == 2) {
      is3d = true;
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        int grc = CSM_OK;
        if (g == 1 && v == 2) ok &= Rigid(y.Sub(), s3->local_pose);
        else if (g == 3) s3->finished = y.Int(v) != 0;
        else if ((g == 4 || g == 5) && v == 2) grc = ParseHybridGrid(y.Sub(), &s3->grids[g - 4]);
        else if (g == 6) Floats(v, y, &s3->histogram);
        else y.Skip(v);
        if (grc != CSM_OK) rc = grc;
      });
    } else if (f == 2 && w == 2) {
      is2d = true;
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        if (g == 1 && v == 2) ok &= Rigid(y.Sub(), s->local_pose);
        else if (g == 3) s->finished = y.Int(v) != 0;
        else if (g == 4 && v == 2) rc = ParseGrid(y.Sub(), s);
        else y.Skip(v);
      });
    } else {
      x.Skip(w);
    }
  });
  if (!ok) return CSM_EINVAL;
  if (rc != CSM_OK) return rc;
  return is2d ? 1 : (is3d ? 2 : 0);
}

// CompressedPointCloud::ConstIterator::ReadNextPoint
// (compressed_point_cloud.cc:79-97).
int Decompress(const std::vector<int32_t>& data, int32_t num_points, std::vector<float>* xyz) {
  // Every point takes one int32 of `data` (plus block headers), so a count
  // beyond data.size() is corrupt: rejected before allocating.
  if (num_points < 0 || static_cast<size_t>(num_points) > data.size()) return CSM_EINVAL;
  xyz->resize(static_cast<size_t>(num_points) * 3);
  size_t in = 0;
  int32_t left_in_block = 0, block[3] = {0, 0, 0};
  constexpr int kBits = 10, kMask = (1 << kBits) - 1;
  constexpr float kPrecision = 0.001f;
  for (int32_t i = 0; i < num_points; ++i) {
    if (left_in_block == 0) {
      if (in + 4 > data.size()) return CSM_EINVAL;
      left_in_block = data[in++];
      for (int a = 0; a < 3; ++a)
        block[a] = static_cast<int32_t>(static_cast<uint32_t>(data[in++]) << kBits);
      if (left_in_block <= 0) return CSM_EINVAL;
    }
    if (in >= data.size()) return CSM_EINVAL;
    --left_in_block;
    const int32_t point = data[in++];
    (*xyz)[3 * i + 0] = static_cast<float>(block[0] + (point & kMask)) * kPrecision;
    (*xyz)[3 * i + 1] = static_cast<float>(block[1] + ((point >> kBits) & kMask)) * kPrecision;
    (*xyz)[3 * i + 2] = static_cast<float>(block[2] + (point >> (2 * kBits))) * kPrecision;
  }
  return CSM_OK;
}

int ParseNode(Reader r, NodeRec* n) {
  bool ok = true;
  int rc = CSM_OK;
  ok &= Fields(r, [&](int f, int w, Reader& x) {
    if (f == 1 && w == 2) {
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        if (g == 1) n->trajectory_id = static_cast<int32_t>(y.Int(v));
        else if (g == 2) n->node_index = static_cast<int32_t>(y.Int(v));
        else y.Skip(v);
      });
    } else if (f == 5 && w == 2) {
      ok &= Fields(x.Sub(), [&](int g, int v, Reader& y) {
        if (g == 1) {
          n->timestamp = y.Int(v);
        } else if (g == 2 && v == 2) {
          ok &= Quat(y.Sub(), n->gravity_alignment);
        } else if (g >= 3 && g <= 5 && v == 2) {
          int32_t num_points = 0;
          std::vector<int32_t> data;
          ok &= Fields(y.Sub(), [&](int h, int u, Reader& z) {
            if (h == 1) num_points = static_cast<int32_t>(z.Int(u));
            else if (h == 3) Int32s(u, z, &data);
            else z.Skip(u);
          });
          const int drc = Decompress(data, num_points, &n->clouds[g - 3]);
          if (drc != CSM_OK) rc = drc;
        } else if (g == 6) {
          Floats(v, y, &n->histogram);
        } else if (g == 7 && v == 2) {
          ok &= Rigid(y.Sub(), n->local_pose);
        } else {
          y.Skip(v);
        }
      });
    } else {
      x.Skip(w);
    }
  });
  if (!ok) return CSM_EINVAL;
  return rc;
}

bool ReadU64(FILE* f, uint64_t* v) {
  uint8_t b[8];
  if (std::fread(b, 1, 8, f) != 8) return false;
  *v = 0;
  for (int i = 0; i < 8; ++i) *v |= static_cast<uint64_t>(b[i]) << (8 * i);
  return true;
}

}  // namespace

struct csm_pbstream {
  std::vector<Submap2DRec> submaps;
  std::vector<Submap3DRec> submaps3d;
  std::vector<NodeRec> nodes;
  uint32_t format_version = 0;
};

extern "C" {

static int PbstreamOpen(const char* path, csm_pbstream** out);

// No exception crosses the C-ABI: an allocation failure while reading is
// CSM_ENOMEM, anything else thrown is a malformed stream.
int csm_pbstream_open(const char* path, csm_pbstream** out) {
  if (!path || !out) return CSM_EINVAL;
  *out = nullptr;
  try {
    return PbstreamOpen(path, out);
  } catch (const std::bad_alloc&) {
    return CSM_ENOMEM;
  } catch (...) {
    return CSM_EINVAL;
  }
}

static int PbstreamOpen(const char* path, csm_pbstream** out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return CSM_EINVAL;
  std::unique_ptr<FILE, int (*)(FILE*)> file_guard(f, &std::fclose);
  std::fseek(f, 0, SEEK_END);
  const long file_size = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::unique_ptr<csm_pbstream> owner(new csm_pbstream());
  csm_pbstream* s = owner.get();
  int rc = CSM_OK;
  uint64_t magic = 0;
  if (!ReadU64(f, &magic) || magic != kMagic) rc = CSM_EINVAL;  // proto_stream.cc:68-73
  std::vector<uint8_t> packed;
  std::string msg;
  bool header = true;
  uint64_t size;
  while (rc == CSM_OK && ReadU64(f, &size)) {
    // One zlib call takes a uInt-sized input; a size past the end of the file
    // is a truncated or corrupt stream (checked before allocating).
    if (size > 0xffffffffull || file_size < 0 ||
        size > static_cast<uint64_t>(file_size - std::ftell(f))) {
      rc = CSM_EINVAL;
      break;
    }
    packed.resize(size);
    if (std::fread(packed.data(), 1, size, f) != size || !Gunzip(packed, &msg)) {
      rc = CSM_EINVAL;
      break;
    }
    Reader r{reinterpret_cast<const uint8_t*>(msg.data()),
             reinterpret_cast<const uint8_t*>(msg.data()) + msg.size()};
    if (header) {  // SerializationHeader {uint32 format_version = 1}
      header = false;
      if (!Fields(r, [&](int fld, int w, Reader& x) {
            if (fld == 1) s->format_version = static_cast<uint32_t>(x.Int(w));
            else x.Skip(w);
          }))
        rc = CSM_EINVAL;
      continue;
    }
    bool ok = Fields(r, [&](int fld, int w, Reader& x) {
      if (rc != CSM_OK) {
        x.Skip(w);
      } else if (fld == 3 && w == 2) {
        Submap2DRec sub;
        Submap3DRec sub3;
        const int got = ParseSubmap(x.Sub(), &sub, &sub3);
        if (got < 0) rc = got;
        else if (got == 1) s->submaps.push_back(std::move(sub));
        else if (got == 2) s->submaps3d.push_back(std::move(sub3));
      } else if (fld == 4 && w == 2) {
        NodeRec node;
        const int got = ParseNode(x.Sub(), &node);
        if (got < 0) rc = got;
        else s->nodes.push_back(std::move(node));
      } else {
        x.Skip(w);
      }
    });
    if (!ok && rc == CSM_OK) rc = CSM_EINVAL;
  }
  file_guard.reset();
  if (rc == CSM_OK && header) rc = CSM_EINVAL;  // no SerializationHeader
  if (rc != CSM_OK) return rc;
  *out = owner.release();
  return CSM_OK;
}

void csm_pbstream_close(csm_pbstream* s) { delete s; }

uint32_t csm_pbstream_format_version(const csm_pbstream* s) { return s ? s->format_version : 0; }

int32_t csm_pbstream_num_submaps2d(const csm_pbstream* s) {
  return s ? static_cast<int32_t>(s->submaps.size()) : 0;
}

int32_t csm_pbstream_num_nodes(const csm_pbstream* s) {
  return s ? static_cast<int32_t>(s->nodes.size()) : 0;
}

int csm_pbstream_submap2d(const csm_pbstream* s, int32_t i, int32_t* ids, csm_map_limits* limits,
                          float* min_max_cc, int32_t* finished, double* local_pose7,
                          uint16_t* cells, int64_t capacity) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->submaps.size())) return CSM_EINVAL;
  const Submap2DRec& r = s->submaps[i];
  if (ids) {
    ids[0] = r.trajectory_id;
    ids[1] = r.submap_index;
  }
  if (limits) *limits = r.limits;
  if (min_max_cc) {
    min_max_cc[0] = r.min_cc;
    min_max_cc[1] = r.max_cc;
  }
  if (finished) *finished = r.finished;
  if (local_pose7) std::memcpy(local_pose7, r.local_pose, sizeof(r.local_pose));
  if (cells) {
    if (capacity < static_cast<int64_t>(r.cells.size())) return CSM_ERANGE;
    std::memcpy(cells, r.cells.data(), r.cells.size() * sizeof(uint16_t));
  }
  return CSM_OK;
}

int csm_pbstream_node(const csm_pbstream* s, int32_t i, int32_t* ids, int64_t* timestamp,
                      double* local_pose7, double* gravity_alignment, float* xyz,
                      int64_t capacity, int32_t* num_points) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->nodes.size())) return CSM_EINVAL;
  const NodeRec& r = s->nodes[i];
  const int64_t n = static_cast<int64_t>(r.clouds[0].size() / 3);
  if (ids) {
    ids[0] = r.trajectory_id;
    ids[1] = r.node_index;
  }
  if (timestamp) *timestamp = r.timestamp;
  if (local_pose7) std::memcpy(local_pose7, r.local_pose, sizeof(r.local_pose));
  if (gravity_alignment) std::memcpy(gravity_alignment, r.gravity_alignment, 4 * sizeof(double));
  if (num_points) *num_points = static_cast<int32_t>(n);
  if (xyz) {
    if (capacity < n) return CSM_ERANGE;
    std::memcpy(xyz, r.clouds[0].data(), r.clouds[0].size() * sizeof(float));
  }
  return CSM_OK;
}

int csm_pbstream_node_cloud(const csm_pbstream* s, int32_t i, int32_t which, float* xyz,
                            int64_t capacity, int32_t* num_points) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->nodes.size()) || which < 0 || which > 2)
    return CSM_EINVAL;
  const std::vector<float>& c = s->nodes[i].clouds[which];
  const int64_t n = static_cast<int64_t>(c.size() / 3);
  if (num_points) *num_points = static_cast<int32_t>(n);
  if (xyz) {
    if (capacity < n) return CSM_ERANGE;
    std::memcpy(xyz, c.data(), c.size() * sizeof(float));
  }
  return CSM_OK;
}

int csm_pbstream_node_histogram(const csm_pbstream* s, int32_t i, float* histogram,
                                int32_t capacity, int32_t* size) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->nodes.size())) return CSM_EINVAL;
  const std::vector<float>& h = s->nodes[i].histogram;
  if (size) *size = static_cast<int32_t>(h.size());
  if (histogram) {
    if (capacity < static_cast<int32_t>(h.size())) return CSM_ERANGE;
    std::memcpy(histogram, h.data(), h.size() * sizeof(float));
  }
  return CSM_OK;
}

int32_t csm_pbstream_num_submaps3d(const csm_pbstream* s) {
  return s ? static_cast<int32_t>(s->submaps3d.size()) : 0;
}

int csm_pbstream_submap3d(const csm_pbstream* s, int32_t i, int32_t* ids, int32_t* finished,
                          double* local_pose7, int64_t* num_cells, int32_t* histogram_size) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->submaps3d.size())) return CSM_EINVAL;
  const Submap3DRec& r = s->submaps3d[i];
  if (ids) {
    ids[0] = r.trajectory_id;
    ids[1] = r.submap_index;
  }
  if (finished) *finished = r.finished;
  if (local_pose7) std::memcpy(local_pose7, r.local_pose, sizeof(r.local_pose));
  if (num_cells) {
    num_cells[0] = static_cast<int64_t>(r.grids[0].values.size());
    num_cells[1] = static_cast<int64_t>(r.grids[1].values.size());
  }
  if (histogram_size) *histogram_size = static_cast<int32_t>(r.histogram.size());
  return CSM_OK;
}

int csm_pbstream_submap3d_grid(const csm_pbstream* s, int32_t i, int32_t which, float* resolution,
                               int32_t* xyz_indices, uint16_t* values, int64_t capacity) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->submaps3d.size()) || which < 0 || which > 1)
    return CSM_EINVAL;
  const HybridGridRec& g = s->submaps3d[i].grids[which];
  if (resolution) *resolution = g.resolution;
  if (xyz_indices || values) {
    if (capacity < static_cast<int64_t>(g.values.size())) return CSM_ERANGE;
    if (xyz_indices) std::memcpy(xyz_indices, g.xyz.data(), g.xyz.size() * sizeof(int32_t));
    if (values) std::memcpy(values, g.values.data(), g.values.size() * sizeof(uint16_t));
  }
  return CSM_OK;
}

int csm_pbstream_submap3d_histogram(const csm_pbstream* s, int32_t i, float* histogram,
                                    int32_t capacity) {
  if (!s || i < 0 || i >= static_cast<int32_t>(s->submaps3d.size())) return CSM_EINVAL;
  const std::vector<float>& h = s->submaps3d[i].histogram;
  if (histogram) {
    if (capacity < static_cast<int32_t>(h.size())) return CSM_ERANGE;
    std::memcpy(histogram, h.data(), h.size() * sizeof(float));
  }
  return CSM_OK;
}

}  // extern "C"
