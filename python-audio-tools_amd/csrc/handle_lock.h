// handle_lock.h — one caller at a time per engine / decoder handle.
//
// The CPython extensions (csrc/ext) and the ctypes shim release the GIL
// around engine calls, and a process shares one engine between its Python
// threads, so two threads may call into the same handle at once.  The
// handle's slots, staging buffers and plan cache are not safe for that
// (DevBuf::ensure may free a buffer another call is using).  Every public
// entry point taking a handle holds the handle's mutex; it is recursive
// because the synchronous calls run the async call and the wait inside.
#pragma once
#include <mutex>

struct HandleLock {
    std::unique_lock<std::recursive_mutex> lk;
    explicit HandleLock(std::recursive_mutex *m)
    {
        if (m)
            lk = std::unique_lock<std::recursive_mutex>(*m);
    }
};

#define ATG_HANDLE_LOCK(h) HandleLock atg_handle_lock_((h) ? &(h)->mu : nullptr)
