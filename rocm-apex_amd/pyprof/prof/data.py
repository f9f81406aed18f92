"""Per-kernel record object of the prof stage (reference apex/pyprof/prof/data.py:3-68).

``Data(kernel)`` takes one record of the parse stage (either this package's parse output or the
reference's NVprof-era dict with ``kShortName`` / ``kLongName`` / ``marker`` / ``mod`` / ``op``
lists) and exposes the reference's attribute names; ``record(mod, op)`` is the normalized dict
the op models (``prof/ops.py``) price, with the argument list decoded from the innermost marker.
"""
import ast


def _last(v, default=""):
    if isinstance(v, (list, tuple)):
        return v[-1] if v else default
    return v if v is not None else default


def _flat(v):
    return str(v).replace(" ", "").replace("(", "").replace(")", "")


class Data(object):
    def __init__(self, kernel):
        self.kernel = kernel
        self.tid = kernel.get("tid", -1)
        self.device = kernel.get("device", 0)
        self.stream = kernel.get("stream", 0)
        self.grid = _flat(kernel.get("grid", ""))
        self.block = _flat(kernel.get("block", ""))
        self.name = str(kernel.get("kShortName", kernel.get("name", ""))).replace(" ", "_")
        self.lName = kernel.get("kLongName", kernel.get("name", ""))
        self.sil = kernel.get("kDuration", 0)  # ns
        self.index = None
        self.argMarker = kernel.get("marker", [])
        self.modMarker = kernel.get("reprMarkers", [])
        self.seqMarker = kernel.get("seqMarker", [])
        self.layer = kernel.get("layer", [])
        self.trace = kernel.get("trace", [])
        self.seqId = kernel.get("seqId", [])
        self.altSeqId = kernel.get("altSeqId", [])
        self.dir = kernel.get("dir", "fprop")
        self.sub = kernel.get("subSeqId", 0)
        self.mod = "na"
        self.op = "na"
        self.params = {"na": "na"}
        self.tc = "na"
        self.flops = 0
        self.bytes = 0

    def args(self):
        """Argument descriptions of the innermost marker (``[]`` when it carries none)."""
        if "args" in self.kernel:
            return self.kernel["args"] or []
        m = _last(self.argMarker, None)
        if isinstance(m, str):
            try:
                m = ast.literal_eval(m)
            except (ValueError, SyntaxError):
                return []
        return (m or {}).get("args", []) if isinstance(m, dict) else []

    def record(self, mod=None, op=None):
        """Normalized record for the op models."""
        return {"mod": _last(mod if mod is not None else self.kernel.get("mod", "")),
                "op": _last(op if op is not None else self.kernel.get("op", "")),
                "args": self.args(), "dir": self.dir, "kName": self.lName,
                "kDuration": self.sil, "tid": self.tid}

    def setParams(self, params):
        """Parameter string of the op (types first-class, everything else ``k=v``), no spaces."""
        out = ""
        for key, value in params.items():
            out += ("{}={},".format(key, value) if "type" not in key else "{},".format(value))
        self.params = out.replace(" ", "")
