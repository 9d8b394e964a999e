// integration/FrameStereo.cc -- optional: Frame::ComputeStereoMatches
// (src/Frame.cc:516-704) on the two extractors' device state.  With this file,
// delete the reference body from src/Frame.cc and define ORB_AMD_GPU_STEREO
// for integration/ORBextractor.cc: the stereo Frame constructor
// (src/Frame.cc:81-93) extracts left and right on two threads, then this
// matches them where the extractions left keypoints, descriptors and both
// pyramids, and copies back only mvuRight / mvDepth.
// The fork's per-candidate debug ofstream (src/Frame.cc:556,652-653) is I/O,
// not algorithm, and is not reproduced.
#include "Frame.h"

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "ORBextractor.h"
#include "orb_abi.h"

namespace ORB_SLAM2 {

void Frame::ComputeStereoMatches() {
  mvuRight = vector<float>(N, -1.0f);  // :519-520
  mvDepth = vector<float>(N, -1.0f);
  struct Handle {
    orb_matcher_t* h = nullptr;
    ~Handle() { orb_matcher_destroy(h); }
  };
  thread_local Handle m;
  // same device as the extractors (integration/ORBextractor.cc): the match
  // runs where both extractions left their pyramids
  const char* dev = std::getenv("ORB_AMD_DEVICE");
  orb_status_t st = m.h ? ORB_OK : orb_matcher_create(dev ? std::atoi(dev) : 0, &m.h);
  int n = 0;
  if (st == ORB_OK)
    st = orb_stereo_match_extracted(m.h, mpORBextractorLeft->gpu(), mpORBextractorRight->gpu(), mbf,
                                    fx, mvuRight.data(), mvDepth.data(), N, &n);
  if (st != ORB_OK || n != N)
    throw std::runtime_error(std::string("Frame::ComputeStereoMatches: ") + orb_status_string(st));
}

}  // namespace ORB_SLAM2
