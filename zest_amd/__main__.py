import sys

from zest_amd.cli import main

sys.exit(main())
