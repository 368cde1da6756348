"""``python -m alluxio_amd.stress <master|worker|client-io|ufs-io|max-throughput> [args]``
(reference: ``bin/alluxio runClass alluxio.stress.cli.<Bench>``); ``report --input .. --output ..``
draws an HTML comparison of result files (GenerateReport).  ``--cluster`` submits the
bench to the job service (StressBenchDefinition) and prints the merged summary."""
import json
import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    bench, rest = argv[0], argv[1:]
    if bench == "report":
        from .report import main as m
        return m(rest)
    if "--cluster" in rest:
        rest.remove("--cluster")
        limit = 0
        if "--cluster-limit" in rest:
            i = rest.index("--cluster-limit")
            limit = int(rest[i + 1])
            del rest[i:i + 2]
        from ..client.context import FileSystemContext
        from ..job import JobClient, StressBenchConfig
        ctx = FileSystemContext()
        status, result, err = JobClient(ctx.master_channel()).run_and_wait(
            StressBenchConfig(bench=bench, args=rest, cluster_limit=limit))
        print(json.dumps({"status": status, "result": result, "error": err}))
        return 0 if status == "COMPLETED" else 1
    if bench == "max-throughput":
        from .max_throughput import main as m
        m(rest)
        return 0
    from . import run_local
    print(json.dumps(run_local(bench, rest)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
