/* mock: see mitsuba/mock.h */
#include <mitsuba/mock.h>
