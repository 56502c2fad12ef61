// convert_icon_main.cpp -- the convert_icon tool (tools/convert_icon/convert_icon.cpp) on
// this backend's netCDF-classic reader:
//
//   convert_icon -hgrid <hg.nc> -hsurf <hs.nc> -hhl [hh.nc*] -data [df.nc*] [-o base]
//                [--var NAME] [--max-layers N] [--no-ic] [--umesh]
//
// Same command line as the reference (parseCommandLine, 121-161).  The reference
// hard-codes convertToIC=false / convertToUMesh=true (22-23) and is normally built
// without UMesh, so as shipped it writes nothing; this tool writes `<base>.ic` (the file
// icon_rt loads) unless --no-ic, and `<base>.umesh` (the UMesh branch, 393-452) with
// --umesh.  --var / --max-layers expose the hard-coded "pres" (308) and maxLayers=5 (24).
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "icon_rt_hip.h"

int main(int argc, char *argv[]) {
  if (argc < 3 || std::string(argv[1]) == "help") {
    fprintf(stderr,
            "Convert DWD ICON data (netCDF classic) to the .ic format icon_rt loads.\n"
            "Usage: convert_icon -hgrid <hg.nc> -hsurf <hs.nc> -hhl [hh.nc*] -data [df.nc*]"
            " [-o base] [--var NAME] [--max-layers N] [--no-ic] [--umesh]\n");
    return 1;
  }
  enum Mode { Hgrid, Hsurf, Hhl, Data, None };
  Mode mode = None;
  std::string hgrid, hsurf, outBase = "out", var = "pres";
  std::vector<std::string> hhl, data;
  int maxLayers = 5;
  bool writeIC = true, writeUMesh = false;
  for (int i = 1; i < argc; ++i) {  // convert_icon.cpp:121-161
    std::string arg = argv[i];
    if (arg[0] != '-') {
      if (mode == Hgrid) hgrid = arg;
      else if (mode == Hsurf) hsurf = arg;
      else if (mode == Hhl) hhl.push_back(arg);
      else if (mode == Data) data.push_back(arg);
      else {
        fprintf(stderr, "Unknown parm: %s\n", argv[i]);
        break;
      }
    } else if (arg == "-hgrid") mode = Hgrid;
    else if (arg == "-hsurf") mode = Hsurf;
    else if (arg == "-hhl") mode = Hhl;
    else if (arg == "-data") mode = Data;
    else if (arg == "-o" && i + 1 < argc) outBase = argv[++i];
    else if (arg == "--var" && i + 1 < argc) var = argv[++i];
    else if (arg == "--max-layers" && i + 1 < argc) maxLayers = atoi(argv[++i]);
    else if (arg == "--no-ic") writeIC = false;
    else if (arg == "--umesh") writeUMesh = true;
  }
  if (hgrid.empty() || hsurf.empty() || hhl.empty()) {
    fprintf(stderr, "Usage: ./convert_icon -hgrid <hg.nc> -hsurf <hs.nc> -hhl [hh.nc*] -data [df.nc*]\n");
    return 1;
  }
  std::vector<const char *> hp, dp;
  for (auto &s : hhl) hp.push_back(s.c_str());
  for (auto &s : data) dp.push_back(s.c_str());
  irt_convert_opts o{hgrid.c_str(), hsurf.c_str(), hp.data(), (int)hp.size(),
                     dp.data(), (int)dp.size(), var.c_str(), maxLayers};
  size_t n = 0;
  if (irt_convert_icon(&o, nullptr, 0, &n)) {
    fprintf(stderr, "convert_icon: %s\n", irt_last_error());
    return 1;
  }
  std::vector<irt_icon_cell> cells(n);
  if (irt_convert_icon(&o, cells.data(), n, &n)) {
    fprintf(stderr, "convert_icon: %s\n", irt_last_error());
    return 1;
  }
  printf("%zu records\n", n);
  if (writeIC) {
    const std::string path = outBase + ".ic";
    if (irt_save_ic(path.c_str(), cells.data(), n)) {
      fprintf(stderr, "convert_icon: %s\n", irt_last_error());
      return 1;
    }
    printf("wrote %s\n", path.c_str());
  }
  if (writeUMesh) {
    const std::string path = outBase + ".umesh";
    size_t nv = 0, nw = 0;
    if (irt_convert_icon_umesh(&o, path.c_str(), &nv, &nw)) {
      fprintf(stderr, "convert_icon: %s\n", irt_last_error());
      return 1;
    }
    printf("%zu\n%zu\nwrote %s\n", nv, nw, path.c_str());  // convert_icon.cpp:444-447
  }
  return 0;
}
