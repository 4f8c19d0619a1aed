// zp_parse_slots.hip — the batch parse kernel with record slots
// (zp_set_record_slots): the same tile code as zp_parse.hip,
// instantiated in its own translation unit so that zp_parse_kernel's code
// is not changed by a second instantiation in the same module.
#define ZP_PARSE_SLOTS_TU 1
#include "zp_parse.hip"
