// parse_solo.hip — the solo / spread parse kernels (k_parse_solo, one image's
// substreams on scalar engines; parse_lanes.hip) as a translation unit of
// their own, so that the lanes kernels and these get the code-generation
// flags each is fastest with (Makefile PARSE_SCHED / SOLO_SCHED; A/B in
// DESIGN 5.11).
#define HG_PARSE_TU 2
#include "parse_lanes.hip"
