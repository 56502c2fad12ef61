// irt_netcdf.h -- a minimal reader for the netCDF *classic* file formats (CDF-1 "classic",
// CDF-2 "64-bit offset", CDF-5 "64-bit data"), enough for convert_icon's use of the netCDF
// C library (tools/convert_icon/convert_icon.cpp:58-118, 187-335): nc_open, nc_inq_dimid +
// nc_inq_dimlen, nc_inq_varid + nc_get_var_int / nc_get_var_double.
//
// The netCDF library itself is not in this image.  The classic format is a big-endian
// header (dims, attributes, variables with their nc_type, shape and file offset) followed
// by the variables' data; record variables (first dim of length 0 = UNLIMITED) interleave
// one slab per record.  netCDF-4 (HDF5) files are detected and refused with a message.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace irt_nc {

enum NcType : int32_t {
  NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6,
  NC_UBYTE = 7, NC_USHORT = 8, NC_UINT = 9, NC_INT64 = 10, NC_UINT64 = 11,
};

struct Dim {
  std::string name;
  uint64_t length = 0;  // 0 = the record (UNLIMITED) dimension
};

struct Var {
  std::string name;
  std::vector<uint32_t> dimids;
  NcType type = NC_BYTE;
  uint64_t vsize = 0;  // bytes per variable (per record for record variables), padded
  uint64_t begin = 0;  // file offset of the data (of record 0 for record variables)
  bool isRecord = false;
};

class File {
 public:
  // Returns false and fills err on failure (missing file, not classic netCDF, truncated).
  bool open(const std::string &path, std::string &err);

  // nc_inq_dimid + nc_inq_dimlen; false if the dimension does not exist.  The record
  // dimension reports the number of records, as nc_inq_dimlen does.
  bool dimLength(const std::string &name, uint64_t &len) const;

  const Var *findVar(const std::string &name) const;

  // Number of values of a variable (product of its dimension lengths, records included).
  static constexpr uint64_t kOverflow = ~0ull;  // numValues of a header whose product overflows
  uint64_t numValues(const Var &v) const;

  // nc_get_var_double / nc_get_var_int: every value of the variable converted to the
  // requested type (C conversion, no _FillValue/scale handling -- as the netCDF library).
  bool readDouble(const Var &v, std::vector<double> &out, std::string &err) const;
  bool readInt(const Var &v, std::vector<int> &out, std::string &err) const;

  int version() const { return version_; }
  const std::vector<Dim> &dims() const { return dims_; }
  const std::vector<Var> &vars() const { return vars_; }

 private:
  bool readRaw(const Var &v, std::vector<uint8_t> &bytes, std::string &err) const;
  std::string path_;
  int version_ = 0;
  uint64_t numrecs_ = 0;
  uint64_t recsize_ = 0;  // bytes per record over all record variables
  std::vector<Dim> dims_;
  std::vector<Var> vars_;
};

size_t typeSize(NcType t);

}  // namespace irt_nc
