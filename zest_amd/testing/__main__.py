from .fakehub import main

raise SystemExit(main())
