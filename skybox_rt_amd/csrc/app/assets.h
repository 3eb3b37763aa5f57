// assets.h -- file lookup of the regression CLIs: graphics::ResolveFilePath
// (sim/common/gfxutil.cpp:348-363) -- the name as given, else in each
// directory of a comma-separated search list; here the list is env
// RT_ASSETS_PATHS (the reference compiles its source directory in as
// ASSETS_PATHS, draw3d/Makefile:14).  `gz`: also accept <name>.gz (scenes
// are committed gzip-compressed where large; the reader inflates them).
#pragma once

#include <sys/stat.h>

#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

namespace rt {

inline std::string ResolveAsset(const std::string& name, bool gz = false) {
  std::vector<std::string> cands = {name};
  if (const char* e = std::getenv("RT_ASSETS_PATHS")) {
    std::stringstream ss(e);
    std::string dir;
    while (std::getline(ss, dir, ','))
      if (!dir.empty()) cands.push_back(dir + "/" + name);
  }
  struct stat sb;
  for (const std::string& c : cands) {
    if (stat(c.c_str(), &sb) == 0) return c;
    if (gz && stat((c + ".gz").c_str(), &sb) == 0) return c + ".gz";
  }
  return name;
}

}  // namespace rt
