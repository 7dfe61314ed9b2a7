// Small helpers shared by the backends.
#include <cctype>
#include <string>

#include "kgs/backend.h"

namespace kgs {

const char* const kEccBlockNames[kEccBlocks] = {"umc", "sdma", "gfx", "mmhub", "athub", "pcie_bif", "hdp",
                                                "xgmi_wafl", "df", "smn", "sem", "mp0", "mp1", "fuse",
                                                "mca", "vcn", "jpeg", "ih", "mpio"};

std::string gpu_type_from_market_name(const std::string& m) {
  // "AMD Instinct MI355 OAM" -> "MI355X"; "AMD Instinct MI300X" -> "MI300X".
  for (size_t i = 0; i + 2 < m.size(); ++i) {
    if (m[i] == 'M' && m[i + 1] == 'I' && std::isdigit(static_cast<unsigned char>(m[i + 2])) &&
        (i == 0 || m[i - 1] == ' ')) {
      size_t j = i + 2;
      while (j < m.size() && std::isdigit(static_cast<unsigned char>(m[j]))) ++j;
      std::string t = m.substr(i, j - i);
      if (j < m.size() && std::isalpha(static_cast<unsigned char>(m[j]))) {
        while (j < m.size() && std::isalnum(static_cast<unsigned char>(m[j]))) t += m[j++];
      } else {
        t += 'X';
      }
      return t;
    }
  }
  return m.empty() ? std::string("unknown") : m;
}

}  // namespace kgs
