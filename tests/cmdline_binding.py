"""ctypes views of struct cmd_line_af_xdp: the reference's (src/cmd_line.h:7-18)
and this build's (pb-af-xdp_amd/host/cmd_line.h, same leading members)."""
import ctypes as C
import ctypes.util

# GCC places the three trailing `unsigned int x : 1` members in the int unit that
# starts at batch_size (byte 18, bits 0-2; struct size 20): declaring them on a
# c_ushort unit reproduces that (checked by test_struct_layout_probe).
REF_FIELDS = [("queue_set", C.c_uint, 1), ("queue", C.c_int), ("no_wake_up", C.c_uint, 1), ("shared_umem", C.c_uint),
              ("batch_size", C.c_ushort), ("skb_mode", C.c_ushort, 1), ("zero_copy", C.c_ushort, 1),
              ("copy", C.c_ushort, 1)]
NAMES = [f[0] for f in REF_FIELDS]


class RefCmd(C.Structure):
    _fields_ = REF_FIELDS


class OurCmd(C.Structure):
    _fields_ = REF_FIELDS + [("gpus", C.c_int), ("gpu_first", C.c_int), ("gpu_batch", C.c_uint64),
                             ("seed_base", C.c_uint64), ("literal_payload", C.c_int), ("single_fold", C.c_int),
                             ("pcap", C.c_char_p), ("tx", C.c_char_p), ("seed_set", C.c_int),
                             ("very_random", C.c_int), ("batch_set", C.c_int), ("umem_frames", C.c_uint32),
                             ("umem_slot", C.c_uint32)]


_libc = C.CDLL(ctypes.util.find_library("c"))


def parse(lib, cls, argv, defaults=None):
    """Run lib's parse_cmd_line_af_xdp on argv (fresh getopt state)."""
    C.c_int.in_dll(_libc, "optind").value = 0
    C.c_int.in_dll(_libc, "opterr").value = 0
    args = [b"pcktbatch"] + [a.encode() for a in argv]
    arr = (C.c_char_p * (len(args) + 1))(*args, None)
    obj = cls()
    if defaults:
        defaults(C.byref(obj))
    else:
        obj.batch_size = 1  # main.c:45-46
    lib.parse_cmd_line_af_xdp(C.byref(obj), len(args), arr)
    return obj


ARGV_CASES = [
    [],
    ["--queue", "3"],
    ["--queue", "-1", "--nowakeup"],
    ["--sharedumem", "--batchsize", "64", "--skb"],
    ["--zerocopy", "--copy", "--queue", "12abc"],
    ["--batchsize", "70000"],
    ["-c", "/etc/x.json", "-z", "--sip", "10.0.0.1", "--queue", "7", "--bogus", "--copy"],
    ["--queue=5", "--batchsize=8", "--nowakeup", "-v"],
    ["--skb", "--gpus", "4", "--queue", "2"],
    ["-v", "--zerocopy", "extra", "--sharedumem"],
]
