// Record sizes shared by the kernels and the C-ABI layer.
#pragma once
#include "sim_params.h"

namespace pbg {
// Pack on explicit inputs (golden-vector parity of the device pack).  Per env the input
// record is float64: [part_xyz (NP+1)*3 | n_parts | quat 4 | pos 3 | vel 3 | jq NO | jqd NO |
// feet_prev NF | feet_new NF | act NA | potential_old | initial_z_in | is_step]; the output
// record: [obs OBS | reward | done | potential | initial_z | feet_out NF].
// HumanoidFlagrun appends to the input [target x, y | flag_timeout | next target x, y] (the
// draw a reposition would take) and to the output [target x, y | flag_timeout].
// HumanoidFlagrunHarder appends to the input [frame | on_ground | crawl_start | crawl_ignored |
// launch draws: angle, speed, jitter 3] and to the output [frame | on_ground | crawl_start |
// crawl_ignored | launched | cube position 3 | cube velocity 3].  The MuJoCo-observation Ant /
// Humanoid append the base angular velocity (3) to the input, Atlas the head part's height.
template <class R>
struct PackRec {
  static constexpr int IN = (R::NP + 1) * 3 + 1 + 4 + 3 + 3 + 2 * R::NO + 2 * R::NF + R::NA + 3 + (R::flagrun ? 5 : 0) +
                            (R::harder ? 9 : 0) + (R::kind == 3 ? 3 : 0) + (R::alive == 13 ? 1 : 0);
  static constexpr int OUT = R::OBS + 4 + R::NF + (R::flagrun ? 3 : 0) + (R::harder ? 11 : 0);
};
template <class R>
struct Records {
  static constexpr int SD = PBG_STATE_WORDS(R::NJ, R::harder);                    // physical state words
  static constexpr int AD = PBG_AUX_RECORD_WORDS(R::NF, R::flagrun, R::harder);  // bookkeeping words
};
}  // namespace pbg
