"""``python -m alluxio_amd <command>`` — the ``bin/alluxio`` equivalent."""
from .cli.main import main

raise SystemExit(main())
