// irt_netcdf.cpp -- netCDF classic (CDF-1/2/5) reader; see irt_netcdf.h.
//
// Header grammar (big-endian; CDF-5 widens counts, dim lengths, dimids and vsize to 64 bits;
// CDF-2 and CDF-5 store `begin` as 64 bits):
//   magic 'C' 'D' 'F' version, numrecs,
//   dim_list  = ABSENT | NC_DIMENSION(0x0A) n {name length}
//   gatt_list = ABSENT | NC_ATTRIBUTE(0x0C) n {name nc_type nvalues values(padded to 4)}
//   var_list  = ABSENT | NC_VARIABLE(0x0B)  n {name ndims dimids vatt_list nc_type vsize begin}
//   name      = n chars (padded to 4)
#include "irt_netcdf.h"

#include <cstdio>
#include <cstring>

namespace irt_nc {

size_t typeSize(NcType t) {
  switch (t) {
    case NC_BYTE: case NC_CHAR: case NC_UBYTE: return 1;
    case NC_SHORT: case NC_USHORT: return 2;
    case NC_INT: case NC_FLOAT: case NC_UINT: return 4;
    case NC_DOUBLE: case NC_INT64: case NC_UINT64: return 8;
  }
  return 0;
}

namespace {

struct Cursor {  // sequential big-endian reads over the file head, refilled on demand
  FILE *f = nullptr;
  std::vector<uint8_t> buf;
  size_t pos = 0;
  bool ok = true;

  bool ensure(size_t n) {
    while (ok && buf.size() - pos < n) {
      uint8_t chunk[65536];
      const size_t got = fread(chunk, 1, sizeof(chunk), f);
      if (got == 0) {
        ok = false;
        break;
      }
      buf.insert(buf.end(), chunk, chunk + got);
    }
    return ok;
  }
  uint64_t be(int bytes) {
    if (!ensure(bytes)) return 0;
    uint64_t v = 0;
    for (int i = 0; i < bytes; ++i) v = (v << 8) | buf[pos + i];
    pos += bytes;
    return v;
  }
  void skip(uint64_t n) {
    if (ensure(n)) pos += n;
  }
  std::string name(int countBytes) {
    const uint64_t n = be(countBytes);
    if (!ok || n > (1u << 20) || !ensure(n)) {
      ok = false;
      return {};
    }
    std::string s(reinterpret_cast<const char *>(&buf[pos]), n);
    pos += n;
    skip((4 - n % 4) % 4);
    return s;
  }
};

constexpr uint32_t kDimension = 0x0A, kVariable = 0x0B, kAttribute = 0x0C;

void skipAttributes(Cursor &c, int cnt) {
  const uint32_t tag = (uint32_t)c.be(4);
  const uint64_t n = c.be(cnt);
  if (tag == 0 && n == 0) return;  // ABSENT
  if (tag != kAttribute) {
    c.ok = false;
    return;
  }
  for (uint64_t i = 0; i < n && c.ok; ++i) {
    c.name(cnt);
    const NcType t = (NcType)c.be(4);
    const uint64_t nv = c.be(cnt);
    uint64_t bytes = 0;
    if (typeSize(t) == 0 || __builtin_mul_overflow(nv, (uint64_t)typeSize(t), &bytes) ||
        bytes > (1ull << 48)) {
      c.ok = false;
      return;
    }
    c.skip(bytes + (4 - bytes % 4) % 4);
  }
}

template <typename T>
T decode(const uint8_t *p, NcType t) {
  uint64_t u = 0;
  const size_t n = typeSize(t);
  for (size_t i = 0; i < n; ++i) u = (u << 8) | p[i];
  switch (t) {
    case NC_BYTE: return (T)(int8_t)u;
    case NC_CHAR: return (T)(uint8_t)u;
    case NC_UBYTE: return (T)(uint8_t)u;
    case NC_SHORT: return (T)(int16_t)u;
    case NC_USHORT: return (T)(uint16_t)u;
    case NC_INT: return (T)(int32_t)u;
    case NC_UINT: return (T)(uint32_t)u;
    case NC_INT64: return (T)(int64_t)u;
    case NC_UINT64: return (T)u;
    case NC_FLOAT: {
      const uint32_t w = (uint32_t)u;
      float f;
      memcpy(&f, &w, 4);
      return (T)f;
    }
    case NC_DOUBLE: {
      double d;
      memcpy(&d, &u, 8);
      return (T)d;
    }
  }
  return T(0);
}

}  // namespace

bool File::open(const std::string &path, std::string &err) {
  path_ = path;
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  Cursor c;
  c.f = f;
  const bool have4 = c.ensure(4);
  if (have4 && c.buf[0] == 0x89 && c.buf[1] == 'H' && c.buf[2] == 'D' && c.buf[3] == 'F') {
    fclose(f);
    err = path + ": netCDF-4/HDF5 file; only the classic formats are read here "
                 "(convert with `nccopy -k cdf5` or `cdo -f nc copy`)";
    return false;
  }
  if (!have4 || c.buf[0] != 'C' || c.buf[1] != 'D' || c.buf[2] != 'F' ||
      (c.buf[3] != 1 && c.buf[3] != 2 && c.buf[3] != 5)) {
    fclose(f);
    err = path + ": not a netCDF classic file";
    return false;
  }
  version_ = c.buf[3];
  c.pos = 4;
  const int cnt = version_ == 5 ? 8 : 4;   // counts, dim lengths, dimids, vsize
  const int off = version_ == 1 ? 4 : 8;   // begin
  numrecs_ = c.be(cnt);
  if (numrecs_ == (version_ == 5 ? ~0ull : 0xFFFFFFFFull)) numrecs_ = 0;  // STREAMING
  // dimensions
  {
    const uint32_t tag = (uint32_t)c.be(4);
    const uint64_t n = c.be(cnt);
    if (!(tag == 0 && n == 0)) {
      if (tag != kDimension) c.ok = false;
      for (uint64_t i = 0; i < n && c.ok; ++i) {
        Dim d;
        d.name = c.name(cnt);
        d.length = c.be(cnt);
        dims_.push_back(d);
      }
    }
  }
  skipAttributes(c, cnt);  // global attributes
  // variables
  {
    const uint32_t tag = (uint32_t)c.be(4);
    const uint64_t n = c.be(cnt);
    if (!(tag == 0 && n == 0)) {
      if (tag != kVariable) c.ok = false;
      for (uint64_t i = 0; i < n && c.ok; ++i) {
        Var v;
        v.name = c.name(cnt);
        const uint64_t nd = c.be(cnt);
        if (nd > 1024) c.ok = false;
        for (uint64_t k = 0; k < nd && c.ok; ++k) {
          const uint64_t id = c.be(cnt);
          if (id >= dims_.size()) c.ok = false;
          v.dimids.push_back((uint32_t)id);
        }
        skipAttributes(c, cnt);
        v.type = (NcType)c.be(4);
        if (typeSize(v.type) == 0) c.ok = false;
        v.vsize = c.be(cnt);
        v.begin = c.be(off);
        v.isRecord = c.ok && !v.dimids.empty() && dims_[v.dimids[0]].length == 0;
        vars_.push_back(v);
      }
    }
  }
  fclose(f);
  if (!c.ok) {
    err = path + ": truncated or malformed netCDF header";
    return false;
  }
  // record size: the sum of the record variables' vsize, except that a lone record
  // variable is not padded (the classic format's special case)
  int numRecVars = 0;
  for (const Var &v : vars_) numRecVars += v.isRecord;
  recsize_ = 0;
  for (const Var &v : vars_) {
    if (!v.isRecord) continue;
    if (numRecVars == 1) {
      uint64_t per = typeSize(v.type);
      for (size_t k = 1; k < v.dimids.size(); ++k) per *= dims_[v.dimids[k]].length;
      recsize_ += per;
    } else {
      recsize_ += v.vsize;
    }
  }
  return true;
}

bool File::dimLength(const std::string &name, uint64_t &len) const {
  for (const Dim &d : dims_)
    if (d.name == name) {
      len = d.length == 0 ? numrecs_ : d.length;
      return true;
    }
  return false;
}

const Var *File::findVar(const std::string &name) const {
  for (const Var &v : vars_)
    if (v.name == name) return &v;
  return nullptr;
}

// The product of the variable's dimension lengths; kOverflow when it does not fit 64 bits
// (a crafted header: no caller's expected count can match it).
uint64_t File::numValues(const Var &v) const {
  uint64_t n = 1;
  for (size_t k = 0; k < v.dimids.size(); ++k) {
    const uint64_t len = (k == 0 && v.isRecord) ? numrecs_ : dims_[v.dimids[k]].length;
    if (__builtin_mul_overflow(n, len, &n)) return kOverflow;
  }
  return n;
}

bool File::readRaw(const Var &v, std::vector<uint8_t> &bytes, std::string &err) const {
  const uint64_t ts = typeSize(v.type);
  const uint64_t total = numValues(v);
  uint64_t size = 0;
  FILE *f = fopen(path_.c_str(), "rb");
  if (!f) {
    err = "cannot open " + path_;
    return false;
  }
  // every byte the reads below store must fit the buffer, and the buffer the file
  fseeko(f, 0, SEEK_END);
  const uint64_t fileBytes = (uint64_t)ftello(f);
  if (total == kOverflow || __builtin_mul_overflow(total, ts, &size) || size > fileBytes) {
    fclose(f);
    err = path_ + ": variable " + v.name + " is larger than the file";
    return false;
  }
  bytes.assign(size, 0);
  bool ok = true;
  if (!v.isRecord) {
    ok = fseeko(f, (off_t)v.begin, SEEK_SET) == 0 &&
         fread(bytes.data(), 1, bytes.size(), f) == bytes.size();
  } else {
    const uint64_t perRec = numrecs_ ? total / numrecs_ * ts : 0;
    for (uint64_t r = 0; r < numrecs_ && ok; ++r) {
      uint64_t at = 0, end = 0;
      ok = !__builtin_mul_overflow(r, perRec, &at) && !__builtin_add_overflow(at, perRec, &end) &&
           end <= bytes.size() && fseeko(f, (off_t)(v.begin + r * recsize_), SEEK_SET) == 0 &&
           fread(bytes.data() + at, 1, perRec, f) == perRec;
    }
  }
  fclose(f);
  if (!ok) err = path_ + ": short read of variable " + v.name;
  return ok;
}

bool File::readDouble(const Var &v, std::vector<double> &out, std::string &err) const {
  std::vector<uint8_t> raw;
  if (!readRaw(v, raw, err)) return false;
  const size_t ts = typeSize(v.type), n = raw.size() / ts;
  out.resize(n);
  for (size_t i = 0; i < n; ++i) out[i] = decode<double>(&raw[i * ts], v.type);
  return true;
}

bool File::readInt(const Var &v, std::vector<int> &out, std::string &err) const {
  std::vector<uint8_t> raw;
  if (!readRaw(v, raw, err)) return false;
  const size_t ts = typeSize(v.type), n = raw.size() / ts;
  out.resize(n);
  for (size_t i = 0; i < n; ++i) out[i] = decode<int>(&raw[i * ts], v.type);
  return true;
}

}  // namespace irt_nc
