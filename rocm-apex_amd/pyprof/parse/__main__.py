import sys

from .parse import main

sys.exit(main())
