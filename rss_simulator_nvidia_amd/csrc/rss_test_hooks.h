// rss_test_hooks.h -- entry points of the TEST-HOOKS build only (librss_toeplitz_hooks.so,
// rss_toeplitz.hip compiled with -DRSS_TEST_HOOKS).  Not part of the product ABI
// (include/rss_toeplitz.h): the product library librss_toeplitz.so exports none of these and
// its hashing path reads no environment; the tests load the hooks build to force the paths a
// launch takes when scratch memory runs short, to fail a launch on purpose and to measure
// the guarded bins' in-flight margin.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// name: "recount" (0 measured, 1 poison every guarded pass, 2 no gate / no recount),
// "range8", "small_lut", "balance", "counts_perm", "resid", "wide" (0 / 1), "prefetch" (-1
// by outputs, 0 / 1 forced), "guard_sleep" (n: a u16 guard's wave sleeps n x s_sleep 127
// before its subtract, so that a heavy-hitter batch really wraps its bin; set on the current
// device), "alloc_fail" (AllocKind bits: those scratch blocks are refused), "fail_launch"
// (k > 0: the k-th IPv4 hash launch from now returns RSS_EIO, e.g. a later chunk of a
// host-memory call).  RSS_EINVAL for an unknown name.
int rss_test_set_option(const char* name, int value);
void rss_test_reset_options(void);

// out[4]: the most adds that landed on a guarded bin between the add that took it to half
// range and the guard's subtract -- [0] the hash pass's u16 bins, [1] the u16 wide passes,
// [2] / [3] the u8 ones (modulo 256) -- since the last reset (reset != 0 zeroes them after
// reading).  Synchronises the device.
int rss_test_guard_margin(uint32_t* out, int reset);

#ifdef __cplusplus
}
#endif
