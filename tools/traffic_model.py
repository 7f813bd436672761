"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE (KB), reported both ways.

MI355X_MICROARCH.md (HBM / rocprofv3 section) says FETCH_SIZE counts 1/2 of the bytes of a *wide
coalesced streaming read* on gfx950, so such reads are doubled.  That correction is applied
only to kernels whose reads are such streams; every engine kernel here reads narrow or
scattered lines, where FETCH_SIZE counts what moved.  Calibration point:
C3's raw FETCH_SIZE, 116-119 MB per launch, equals the 117 MB delay schedule the exec kernel
reads -- undoubled.

Per kernel: (streaming, reason).  Kernels not listed: not streaming."""

KERNEL_READS = {
    # batch engine: each lane (or each 8-lane instance segment) stages ITS instance's delay row
    # (112 B on C3), and the slot map scatters the instances of a wave
    "cl_exec_kernel": (False, "per-instance delay rows of 112 B (C3) / 64 B (C2), scattered by the slot map"),
    "clsnap_lanes": (False, "per-lane delay rows, one 16-B load per lane per step, scattered by the slot map"),
    # graph engine: per-node and per-channel records at data-dependent addresses
    "k_pick": (False, "one ring head and one route/tokens/cursor line per popping channel, data-dependent"),
    "k_marker": (False, "per-receiver state lines of the channels that delivered markers"),
    "k_push": (False, "ring tails and head words of the pushing channels"),
    "k_scan": (False, "block sums over a few KB"),
    "k_hostops": (False, "a handful of node records"),
    "k_tally": (False, "per-block counters"),
    "k_reset": (False, "writes only"),
    "k_sn_reset": (False, "writes only"),
}


def streaming(kernel_name):
    for k, (s, _) in KERNEL_READS.items():
        if k in kernel_name:
            return s
    return False


def reason(kernel_name):
    for k, (_, r) in KERNEL_READS.items():
        if k in kernel_name:
            return r
    return "not a wide coalesced stream"


def bytes_both(fetch_kb, write_kb, is_streaming):
    """(raw, corrected, justified) bytes."""
    raw = (fetch_kb + write_kb) * 1024
    corrected = (2 * fetch_kb + write_kb) * 1024
    return raw, corrected, corrected if is_streaming else raw
