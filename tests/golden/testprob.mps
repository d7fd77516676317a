* TESTPROB: the example of the MPS format description (fixed format).
* min XONE + 2 YTWO + 3 ZTHREE  s.t. LIM1: XONE + YTWO <= 4,
* LIM2: XONE + ZTHREE >= 1, MYEQN: -YTWO + ZTHREE = 7,
* 0 <= XONE <= 4, -1 <= YTWO <= 1, ZTHREE >= 0.
NAME          TESTPROB
ROWS
 N  COST
 L  LIM1
 G  LIM2
 E  MYEQN
COLUMNS
    XONE      COST         1   LIM1         1
    XONE      LIM2         1
    YTWO      COST         2   LIM1         1
    YTWO      MYEQN       -1
    ZTHREE    COST         3   LIM2         1
    ZTHREE    MYEQN        1
RHS
    RHS1      LIM1         4   LIM2         1
    RHS1      MYEQN        7
BOUNDS
 UP BND1      XONE         4
 LO BND1      YTWO        -1
 UP BND1      YTWO         1
ENDATA
